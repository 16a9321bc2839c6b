// fetchcal.hip — calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 against known byte
// counts, per access width (MI355X_MICROARCH.md, HBM section: "Other access widths are uncalibrated:
// calibrate on a known byte count in your own access pattern").  Each kernel streams a 1 GiB buffer
// (4x the 256 MiB Infinity Cache, so every byte comes from HBM) once, coalesced, with one access width
// per launch: the loads of the pair kernels are 16-B records (k_sweep<2>'s ring), 8-B entries
// (k_sweep_pairs' windows, k_sweep_scatter's slots), 4-B columns and 1-B read lengths.  The stores:
// 8-B entries, streaming and in short runs at scattered places (the grouping's bucket segments).
//   hipcc -O3 --offload-arch=gfx950 -o fetchcal fetchcal.hip
//   rocprofv3 --pmc FETCH_SIZE -- ./fetchcal    (then WRITE_SIZE; tools/fetch_calibration.py)
// Prints one JSON line: the kernels' names and their algorithmic read / write bytes.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));           \
      std::exit(1);                                                                           \
    }                                                                                         \
  } while (0)

template <typename T>
__device__ __forceinline__ unsigned fold(const T& v) {
  const unsigned* w = reinterpret_cast<const unsigned*>(&v);
  unsigned x = 0;
  for (unsigned k = 0; k < (sizeof(T) + 3) / 4; ++k) x ^= w[k];
  return x;
}
template <>
__device__ __forceinline__ unsigned fold<unsigned char>(const unsigned char& v) { return v; }

// every element read once, grid-stride; one word per thread written (a negligible 4 B per thread)
template <typename T>
__device__ __forceinline__ void read_all(const T* __restrict__ src, long long n, unsigned* __restrict__ sink) {
  unsigned acc = 0;
  const long long stride = static_cast<long long>(gridDim.x) * blockDim.x;
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < n; i += stride)
    acc = acc * 31u + fold(src[i]);
  if (acc == 0x9E3779B9u) sink[blockIdx.x * blockDim.x + threadIdx.x] = acc;   // practically never taken
}

template <typename T>
__device__ __forceinline__ void write_all(T* __restrict__ dst, long long n) {
  const long long stride = static_cast<long long>(gridDim.x) * blockDim.x;
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < n; i += stride) {
    T v;
    unsigned char* b = reinterpret_cast<unsigned char*>(&v);
    for (unsigned k = 0; k < sizeof(T); ++k) b[k] = static_cast<unsigned char>(i + k);
    dst[i] = v;
  }
}

__global__ __launch_bounds__(256) void k_read16(const uint4* s, long long n, unsigned* k) { read_all(s, n, k); }
__global__ __launch_bounds__(256) void k_read8(const uint2* s, long long n, unsigned* k) { read_all(s, n, k); }
__global__ __launch_bounds__(256) void k_read4(const unsigned* s, long long n, unsigned* k) { read_all(s, n, k); }
__global__ __launch_bounds__(256) void k_read1(const unsigned char* s, long long n, unsigned* k) { read_all(s, n, k); }
__global__ __launch_bounds__(256) void k_write16(uint4* d, long long n) { write_all(d, n); }
__global__ __launch_bounds__(256) void k_write8(unsigned long long* d, long long n) { write_all(d, n); }

// 8-B stores in runs of `run` consecutive elements at segment starts spread over the buffer (the
// grouping scatter's pattern: each wave's lanes write runs into ~1024 bucket segments); every element of
// the buffer is written exactly once
__global__ __launch_bounds__(256) void k_write8_runs(unsigned long long* __restrict__ dst, long long n, int run,
                                                    long long n_seg) {
  const long long stride = static_cast<long long>(gridDim.x) * blockDim.x;
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < n; i += stride) {
    const long long r = i / run, o = i % run;
    // run r goes to segment (r mod n_seg), position r / n_seg inside it
    const long long seg = r % n_seg, slot = r / n_seg;
    const long long per = n / n_seg;
    const long long at = seg * per + slot * run + o;
    if (at < n) dst[at] = static_cast<unsigned long long>(i);
  }
}

int main() {
  const long long bytes = 1ll << 30;
  void* buf = nullptr;
  unsigned* sink = nullptr;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&sink, 1 << 24));
  CK(hipMemset(buf, 1, bytes));
  CK(hipDeviceSynchronize());
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int grid = cus * 8;
  std::printf("{\"buffer_bytes\": %lld, \"kernels\": {", bytes);
  // reads: 16, 8, 4, 1 B per lane; writes: 16, 8 B per lane streaming, 8 B in runs of 6 over 1024 segments
  k_read16<<<grid, 256>>>(static_cast<const uint4*>(buf), bytes / 16, sink);
  k_read8<<<grid, 256>>>(static_cast<const uint2*>(buf), bytes / 8, sink);
  k_read4<<<grid, 256>>>(static_cast<const unsigned*>(buf), bytes / 4, sink);
  k_read1<<<grid, 256>>>(static_cast<const unsigned char*>(buf), bytes, sink);
  k_write16<<<grid, 256>>>(static_cast<uint4*>(buf), bytes / 16);
  k_write8<<<grid, 256>>>(static_cast<unsigned long long*>(buf), bytes / 8);
  k_write8_runs<<<grid, 256>>>(static_cast<unsigned long long*>(buf), bytes / 8, 6, 1024);
  std::printf("\"k_read16\": {\"width\": 16, \"read\": %lld, \"write\": 0}, ", bytes);
  std::printf("\"k_read8\": {\"width\": 8, \"read\": %lld, \"write\": 0}, ", bytes);
  std::printf("\"k_read4\": {\"width\": 4, \"read\": %lld, \"write\": 0}, ", bytes);
  std::printf("\"k_read1\": {\"width\": 1, \"read\": %lld, \"write\": 0}, ", bytes);
  std::printf("\"k_write16\": {\"width\": 16, \"read\": 0, \"write\": %lld}, ", bytes);
  std::printf("\"k_write8\": {\"width\": 8, \"read\": 0, \"write\": %lld}, ", bytes);
  std::printf("\"k_write8_runs\": {\"width\": 8, \"run\": 6, \"segments\": 1024, \"read\": 0, \"write\": %lld}", bytes);
  std::printf("}}\n");
  CK(hipDeviceSynchronize());
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
