// Native host -> HBM staging of a file (SDFS shard replica) for HbmStager.
//
// The Python path (runtime/data.py HbmStager._stage_file) ran its parallel
// preadv calls as thread-pool futures: every call re-acquires the GIL when it
// returns, and with the node's round thread polling in Python those re-acquires
// waited out the interpreter's switch interval -- a 75 MB shard took ~5.5 ms
// to stage during forwards against ~2.2 ms alone (profiles/r5_sdfs_trace*.json,
// tools/overlap_probe.py).  Here the whole shard is staged with the GIL
// released: for each piece of the file, nthreads std::threads fill one pinned
// buffer with pread(2) while the DMA engine copies the previous piece out of the
// other (hipMemcpyAsync on the caller's side stream), a buffer reused only after
// the event of its last copy.  Returns once every copy out of the pinned
// buffers has completed (the buffers are free for the next call).
#include <ATen/hip/HIPContext.h>
#include <fcntl.h>
#include <torch/extension.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cerrno>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include <hip/hip_runtime.h>

namespace idunno {

namespace {

void check_hip(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, what, ": ", hipGetErrorString(e));
}

// fill dst[0, n) from file offset off with up to nthreads parallel pread(2)
// calls; returns false on a short read / error (errno kept in err)
bool pread_parallel(int fd, char* dst, size_t n, size_t off, int nthreads, int* err) {
  const size_t min_part = 4u << 20;
  int nt = (int)std::max<size_t>(1, std::min<size_t>((size_t)nthreads, n / min_part));
  const size_t part = (n + nt - 1) / nt;
  std::atomic<int> bad{0};
  auto work = [&](int i) {
    size_t a = (size_t)i * part, b = std::min(n, a + part);
    while (a < b) {
      const ssize_t k = ::pread(fd, dst + a, b - a, (off_t)(off + a));
      if (k <= 0) {
        if (k < 0 && errno == EINTR) continue;
        bad.store(k < 0 ? errno : EIO);
        return;
      }
      a += (size_t)k;
    }
  };
  if (nt == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    th.reserve(nt - 1);
    for (int i = 1; i < nt; ++i) th.emplace_back(work, i);
    work(0);
    for (auto& t : th) t.join();
  }
  *err = bad.load();
  return *err == 0;
}

}  // namespace

// out: contiguous uint8 device tensor of the file's first out.numel() bytes;
// pinned: >= 1 pinned host uint8 buffers (ping-pong); stream: the side stream
// (hipStream_t as an integer, torch.cuda.Stream.cuda_stream)
// Returns (seconds in pread, seconds waiting for a pinned buffer's previous copy,
// seconds waiting for the last copies at the end).
std::vector<double> stage_file_native(const std::string& path, torch::Tensor out, std::vector<torch::Tensor> pinned,
                                      int64_t stream, int64_t nthreads) {
  TORCH_CHECK(out.is_cuda() && out.is_contiguous() && out.scalar_type() == torch::kUInt8, "out: contiguous uint8 GPU");
  TORCH_CHECK(!pinned.empty(), "no pinned buffers");
  size_t step = (size_t)-1;
  for (auto& p : pinned) {
    TORCH_CHECK(p.is_pinned() && p.is_contiguous() && p.scalar_type() == torch::kUInt8, "pinned: uint8 pinned host");
    step = std::min(step, (size_t)p.numel());
  }
  TORCH_CHECK(step > 0, "empty pinned buffer");
  const size_t nbytes = (size_t)out.numel();
  char* dst = reinterpret_cast<char*>(out.data_ptr());
  const int nb = (int)pinned.size();
  std::vector<char*> pb(nb);
  for (int b = 0; b < nb; ++b) pb[b] = reinterpret_cast<char*>(pinned[b].data_ptr());
  auto st = reinterpret_cast<hipStream_t>(stream);
  int dev = out.get_device();

  pybind11::gil_scoped_release nogil;
  check_hip(hipSetDevice(dev), "hipSetDevice");
  const int fd = ::open(path.c_str(), O_RDONLY);
  TORCH_CHECK(fd >= 0, "open ", path, ": ", std::strerror(errno));
  std::vector<hipEvent_t> done(nb, nullptr);
  std::string fail;
  bool issued = false;                       // some copy out of a pinned buffer was queued
  // every exit path (a read or HIP error included) closes the file, waits until no
  // copy out of the pinned buffers is in flight -- the caller reuses them at once --
  // and destroys the events; the first error is reported only after that
  struct Tail {
    int fd;
    std::vector<hipEvent_t>& done;
    const std::string& fail;
    const bool& issued;
    hipStream_t st;
    ~Tail() {
      ::close(fd);
      if (!fail.empty() && issued) (void)hipStreamSynchronize(st);   // an event may be missing
      for (auto e : done) {
        if (e != nullptr) {
          (void)hipEventSynchronize(e);
          (void)hipEventDestroy(e);
        }
      }
    }
  };
  auto hip_ok = [&](hipError_t e, const char* what) {
    if (e != hipSuccess && fail.empty()) fail = std::string(what) + ": " + hipGetErrorString(e);
    return e == hipSuccess;
  };
  using clk = std::chrono::steady_clock;
  double t_read = 0, t_wait = 0, t_tail = 0;
  auto secs = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); };
  clk::time_point t3;
  {
    Tail tail{fd, done, fail, issued, st};
    for (size_t off = 0, i = 0; off < nbytes; off += step, ++i) {
      const int b = (int)(i % nb);
      const size_t n = std::min(step, nbytes - off);
      auto t0 = clk::now();
      if (done[b] != nullptr && !hip_ok(hipEventSynchronize(done[b]), "hipEventSynchronize")) break;
      auto t1 = clk::now();
      int err = 0;
      const bool ok = pread_parallel(fd, pb[b], n, off, (int)nthreads, &err);
      auto t2 = clk::now();
      t_wait += secs(t0, t1);
      t_read += secs(t1, t2);
      if (!ok) {
        fail = std::string("read ") + path + ": " + std::strerror(err);
        break;
      }
      if (!hip_ok(hipMemcpyAsync(dst + off, pb[b], n, hipMemcpyHostToDevice, st), "hipMemcpyAsync")) break;
      issued = true;
      if (done[b] == nullptr &&
          !hip_ok(hipEventCreateWithFlags(&done[b], hipEventDisableTiming), "hipEventCreate")) {
        done[b] = nullptr;
        break;
      }
      if (!hip_ok(hipEventRecord(done[b], st), "hipEventRecord")) break;
    }
    t3 = clk::now();
  }                                          // ~Tail: the last copies out of the pinned buffers
  t_tail = secs(t3, clk::now());
  TORCH_CHECK(fail.empty(), fail);
  return {t_read, t_wait, t_tail};
}

}  // namespace idunno
