// Host-side launch helpers shared by the kernel TUs.
//
// Per-device state: one process may drive several GPUs (node threads of a
// LocalCluster, tests), and several host threads may race on a kernel's first
// launch.  Both the dynamic-LDS opt-in (hipFuncSetAttribute) and the CU count
// are therefore kept per (kernel, device) under a lock, never in a plain
// function-local `static bool`.
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>
#include <set>
#include <utility>

namespace idunno {

inline int current_device() {
  int dev = 0;
  (void)hipGetDevice(&dev);
  return dev;
}

// Opt kernel `kern` into `bytes` of dynamic LDS on the current device (needed
// above 64 KiB); idempotent and thread-safe, once per (kernel, device).
inline void ensure_lds_attr(const void* kern, int bytes) {
  static std::mutex mu;
  static auto* done = new std::set<std::pair<const void*, int>>();
  const int dev = current_device();
  std::lock_guard<std::mutex> lk(mu);
  if (done->insert({kern, dev}).second)
    (void)hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

// CU count of the current device (cached per device; 256 on MI355X).
inline int device_cu_count() {
  static std::mutex mu;
  static int cus[64] = {0};
  const int dev = current_device();
  if (dev < 0 || dev >= 64) return 256;
  std::lock_guard<std::mutex> lk(mu);
  if (cus[dev] <= 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}

}  // namespace idunno
