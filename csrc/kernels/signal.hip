// Stream-position signal for the data-parallel comm thread (parallel/ddp.py).
//
// The segmented data-parallel step (train/graphs.py) used to end a HIP graph
// at every all-reduce issue point and record an event there, so the host comm
// thread could learn when the compute stream had produced the span's
// gradients. On MI355X that boundary costs the compute stream ~11 us (graph
// boundary ~5 us + event record ~6 us, scripts/graph_boundary_lab.py) at each
// of the step's issue points. Instead, a one-wave kernel captured INSIDE the
// graph at the issue point bumps a device counter and publishes it to a
// fine-grained (coherent) host word with a system-scope store; the comm
// thread spins on that word (signal_wait in bindings.cpp, GIL released) and issues the
// collective once it reaches the value it expects. No graph boundary, no
// event. Kernels of one stream run in order and each ends with a device-wide
// release, so when the signal kernel runs every gradient before it is final
// in memory; the store itself needs no release of its own (a release fence
// would first write back this XCD's L2, and this kernel has nothing to
// publish). A launch costs ~4.6 us of stream time (profiles/r6/dp_signal_issue.txt).
#include <hip/hip_runtime.h>

#include <cstdint>

namespace tdg {

__global__ void __launch_bounds__(64) stream_signal_kernel(unsigned long long* cnt,
                                                           unsigned long long* host) {
  if (threadIdx.x != 0) return;
  const unsigned long long v = cnt[0] + 1ull;
  cnt[0] = v;
  __hip_atomic_store(host, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace tdg

extern "C" {

// host: coherent pinned word (host pointer), dhost: its device address,
// cnt: device counter. Returns 0 on success.
int tdg_signal_create(unsigned long long** host, unsigned long long** dhost,
                      unsigned long long** cnt) {
  void* h = nullptr;
  if (hipHostMalloc(&h, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return -1;
  *static_cast<volatile unsigned long long*>(h) = 0;
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) return -2;
  void* c = nullptr;
  if (hipMalloc(&c, 64) != hipSuccess) return -3;
  if (hipMemset(c, 0, 64) != hipSuccess) return -4;
  if (hipDeviceSynchronize() != hipSuccess) return -5;
  *host = static_cast<unsigned long long*>(h);
  *dhost = static_cast<unsigned long long*>(d);
  *cnt = static_cast<unsigned long long*>(c);
  return 0;
}

int tdg_signal_emit(unsigned long long* cnt, unsigned long long* dhost, hipStream_t st) {
  hipLaunchKernelGGL(tdg::stream_signal_kernel, dim3(1), dim3(64), 0, st, cnt, dhost);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // extern "C"
