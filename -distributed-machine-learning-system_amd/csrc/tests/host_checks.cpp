// Host-side checks of the kernels' index math, built with host AddressSanitizer +
// UndefinedBehaviorSanitizer (GPU sanitizers are not available on
// this pool, so the native code's sanitizer coverage is its host-callable part).
// Exercises the exact __host__ __device__ functions the kernels inline
// (csrc/tile_math.h):
//   * xcd_remap is a bijection on [0, nwg) for every grid size up to 20000 and
//     maps each XCD's round-robin share onto one contiguous logical range;
//   * every LDS swizzle permutes the 16-byte chunks of a row, and every
//     ds_read_b128 lane group of a 16x16x32 fragment read touches 16 distinct
//     16-byte bank slots (MI355X_MICROARCH.md §LDS).
// Build + run: tests/test_host_checks.py.  Exit status = number of failures.
#include <cstdio>
#include <vector>

#include "../tile_math.h"

using namespace idunno;

static int g_fail = 0;
#define CHECK(c, ...)                                  \
  do {                                                 \
    if (!(c)) {                                        \
      if (g_fail++ < 20) std::printf(__VA_ARGS__);     \
    }                                                  \
  } while (0)

// ds_read_b128 serves a wave64 in four groups of 16 lanes, one LDS cycle each
static const int kGroups[4][16] = {
    {0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
    {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
    {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
    {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63},
};

static void check_groups_partition() {
  std::vector<int> seen(64, 0);
  for (auto& g : kGroups)
    for (int l : g) seen[l]++;
  for (int l = 0; l < 64; ++l) CHECK(seen[l] == 1, "lane %d in %d groups\n", l, seen[l]);
}

static void check_xcd_remap() {
  for (int nwg = 1; nwg <= 20000; ++nwg) {
    std::vector<unsigned char> hit(nwg, 0);
    for (int o = 0; o < nwg; ++o) {
      const int t = xcd_remap(o, nwg);
      CHECK(t >= 0 && t < nwg, "xcd_remap(%d, %d) = %d out of range\n", o, nwg, t);
      if (t >= 0 && t < nwg) {
        CHECK(!hit[t], "xcd_remap(., %d) hits %d twice\n", nwg, t);
        hit[t] = 1;
      }
    }
    if (nwg < 16) continue;
    // the workgroups one XCD runs (orig % 8 == x) cover one contiguous logical range
    for (int x = 0; x < 8; ++x) {
      int lo = nwg, hi = -1, n = 0;
      for (int o = x; o < nwg; o += 8, ++n) {
        const int t = xcd_remap(o, nwg);
        lo = t < lo ? t : lo;
        hi = t > hi ? t : hi;
      }
      CHECK(hi - lo + 1 == n, "nwg %d xcd %d: logical range [%d, %d] holds %d tiles\n", nwg, x, lo, hi, n);
    }
  }
}

template <typename F>
static void check_swizzle(const char* name, int cpr, F swz) {
  for (int row = 0; row < 256; ++row) {
    std::vector<int> hit(cpr, 0);
    for (int c = 0; c < cpr; ++c) {
      const int s = c ^ swz(row);
      CHECK(s >= 0 && s < cpr, "%s row %d chunk %d -> %d out of row\n", name, row, c, s);
      if (s >= 0 && s < cpr) hit[s]++;
    }
    for (int s = 0; s < cpr; ++s) CHECK(hit[s] == 1, "%s row %d: slot %d hit %d times\n", name, row, s, hit[s]);
  }
  // 16x16x32 fragment read: lane l reads row base + (l & 15), chunk (l >> 4) + 4 kk
  for (int base = 0; base < 256; base += 16)
    for (int kk = 0; kk < cpr / 4; ++kk)
      for (auto& g : kGroups) {
        int used[16] = {0};
        for (int l : g) {
          const int row = base + (l & 15), chunk = (l >> 4) + 4 * kk;
          const int addr = row * cpr * 16 + ((chunk ^ swz(row)) << 4);
          used[(addr / 16) % 16]++;
        }
        for (int s = 0; s < 16; ++s)
          CHECK(used[s] == 1, "%s cpr %d base %d kk %d: bank slot %d used %d times\n", name, cpr, base, kk, s,
                used[s]);
      }
}

// conv_wino_f32 raw patch read: lane l (tile l & 15 of a row segment starting at
// pixel p0, channel group g = l >> 4) reads pixel p0 + (l & 15) (+1 for the odd
// patch columns), chunk g ^ wino_raw_swz(pixel) of a 64-byte pixel slot
static void check_wino_raw() {
  for (int p0 = 0; p0 < 64; ++p0)
    for (int shift = 0; shift < 2; ++shift)
      for (auto& grp : kGroups) {
        int used[16] = {0};
        for (int l : grp) {
          const int p = p0 + (l & 15) + shift, g = l >> 4;
          const int addr = p * 64 + ((g ^ wino_raw_swz(p)) << 4);
          used[(addr / 16) % 16]++;
        }
        for (int s = 0; s < 16; ++s)
          CHECK(used[s] == 1, "wino raw p0 %d shift %d: bank slot %d used %d times\n", p0, shift, s, used[s]);
      }
  for (int p = 0; p < 256; ++p) {   // a permutation of the pixel's 4 chunks
    int hit[4] = {0};
    for (int g = 0; g < 4; ++g) hit[g ^ wino_raw_swz(p)]++;
    for (int c = 0; c < 4; ++c) CHECK(hit[c] == 1, "wino raw pixel %d: chunk %d hit %d times\n", p, c, hit[c]);
  }
}

int main() {
  check_groups_partition();
  check_xcd_remap();
  check_swizzle("conv_glds swz_r", 8, [](int r) { return swz_r(r, 8); });
  check_swizzle("conv_glds swz_r", 4, [](int r) { return swz_r(r, 4); });
  check_swizzle("conv3x3_c64 c64_swz", 8, [](int r) { return c64_swz(r); });
  check_wino_raw();
  std::printf("host_checks: %d failure(s)\n", g_fail);
  return g_fail ? 1 : 0;
}
