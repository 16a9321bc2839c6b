// Grouping-sort microbenchmark: n u64 match entries (A in the top 25 bits), sorted on A's bits only,
// with rocprim onesweep at several radix widths.  Usage: ./sortbench [n] [reads]
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <unsigned Bits, unsigned Ipt>
using Cfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 12>, rocprim::kernel_config<256, Ipt>, Bits>>;

template <class C>
float run(const unsigned long long* in, unsigned long long* out, size_t n, int b0, int b1, const char* name) {
  size_t tb = 0;
  CK(rocprim::radix_sort_keys<C>(nullptr, tb, in, out, n, b0, b1, 0));
  void* tmp; CK(hipMalloc(&tmp, tb));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int w = 0; w < 2; ++w) CK(rocprim::radix_sort_keys<C>(tmp, tb, in, out, n, b0, b1, 0));
  CK(hipDeviceSynchronize());
  const int reps = 10;
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r) CK(rocprim::radix_sort_keys<C>(tmp, tb, in, out, n, b0, b1, 0));
  CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  printf("%-28s %8.1f us  (temp %zu MB)\n", name, 1000.0f * ms / reps, tb >> 20);
  CK(hipFree(tmp));
  return ms / reps;
}

int main(int argc, char** argv) {
  size_t n = argc > 1 ? atoll(argv[1]) : 18000000;
  long long reads = argc > 2 ? atoll(argv[2]) : 1000000;
  int bits = 1; while ((1ll << bits) < reads) ++bits;
  std::vector<unsigned long long> h(n);
  std::mt19937_64 rng(1);
  for (auto& x : h) x = ((rng() % reads) << 39) | (rng() & ((1ull << 39) - 1));
  unsigned long long *in, *out;
  CK(hipMalloc(&in, n * 8)); CK(hipMalloc(&out, n * 8));
  CK(hipMemcpy(in, h.data(), n * 8, hipMemcpyHostToDevice));
  printf("n = %zu, reads = %lld, A bits = %d\n", n, reads, bits);
  run<rocprim::default_config>(in, out, n, 39, 39 + bits, "default");
  run<Cfg<8, 12>>(in, out, n, 39, 39 + bits, "onesweep 8 bits");
  run<Cfg<8, 16>>(in, out, n, 39, 39 + bits, "onesweep 8 bits, 16 ipt");
  run<rocprim::default_config>(in, out, n, 39 + 6, 39 + bits, "default, A>>6");
  run<Cfg<7, 16>>(in, out, n, 39 + 6, 39 + bits, "onesweep 7 bits 16 ipt, A>>6");
  run<Cfg<7, 12>>(in, out, n, 39 + 6, 39 + bits, "onesweep 7 bits, A>>6");
  // plain copy of the same bytes, for the HBM reference
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < 10; ++r) CK(hipMemcpyAsync(out, in, n * 8, hipMemcpyDeviceToDevice, 0));
  CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  printf("%-28s %8.1f us\n", "copy (read + write once)", 100.0f * ms);
  return 0;
}
