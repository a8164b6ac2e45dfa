// W3 isolation (DESIGN.md "Round-5 changes"): the smallest program that makes
// one cooperative launch and exits.  Run once under
//   rocprofv3 --kernel-trace -- kmldpc_amd/bin/coop_exit [n]
// If it dies in exit() like the library's PEG8064 runs (SIGSEGV inside
// libhsa-runtime64's shutdown), the fault belongs to the runtime / profiler
// teardown, not to kmldpc_amd.  n > 0: n cooperative launches (default 1);
// n < 0: |n| plain launches of the same kernel (the control).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ void empty_kernel(int *out) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && out) out[0] = 1;
}

int main(int argc, char **argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 1;
  int *d = nullptr;
  if (hipMalloc(&d, sizeof(int)) != hipSuccess) return 2;
  void *args[] = {&d};
  for (int i = 0; i < (n < 0 ? -n : n); ++i) {
    const hipError_t e = n > 0 ? hipLaunchCooperativeKernel((const void *)empty_kernel, dim3(256), dim3(64), args, 0, 0)
                               : hipLaunchKernel((const void *)empty_kernel, dim3(256), dim3(64), args, 0, 0);
    if (e != hipSuccess) {
      fprintf(stderr, "launch %d: %s\n", i, hipGetErrorString(e));
      return 3;
    }
  }
  int h = 0;
  if (hipMemcpy(&h, d, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return 4;
  (void)hipFree(d);
  printf("%s launches: %d, flag %d; exiting\n", n > 0 ? "cooperative" : "plain", n < 0 ? -n : n, h);
  return 0;
}
