// PCIe read probe (experiments only, not product code): how fast can a gfx950 kernel read host
// memory the GPU maps, in the access patterns rtn_stage_gather uses? Frames sit in 2176-B
// buffers of a pinned pool in shuffled order (a DPDK mempool after churn); the kernels read B
// bytes of each frame through a pointer array and write them to HBM.
//
//   hipcc --offload-arch=gfx950 -O3 tools/pcie_probe.hip -o tools/_ab/pcie_probe
//   tools/_ab/pcie_probe [frames]
//
// Prints one JSON line per pattern: Mframes/s, GB/s of payload, read requests/s.
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) v4u* gv4u;

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

// Q lanes per frame (16 B each: B = 16 Q bytes per frame), L loads in flight per lane: one wave
// covers L * 64 / Q frames.
template <int Q, int L>
__global__ void __launch_bounds__(256) gather(const unsigned long long* ptrs, unsigned n, v4u* out) {
  const unsigned lane = threadIdx.x & 63u;
  const unsigned wave = blockIdx.x * 4u + (threadIdx.x >> 6);
  constexpr unsigned FPW = L * 64 / Q;  // frames per wave
  const unsigned base = wave * FPW;
  if (base >= n) return;
  v4u x[L];
#pragma unroll
  for (int k = 0; k < L; ++k) {
    const unsigned f = base + k * (64 / Q) + lane / Q;
    const unsigned fc = f < n ? f : n - 1;
    x[k] = *reinterpret_cast<gv4u>(ptrs[fc] + 16u * (lane % Q));
  }
#pragma unroll
  for (int k = 0; k < L; ++k) {
    const unsigned f = base + k * (64 / Q) + lane / Q;
    if (f < n) out[(size_t)f * Q + lane % Q] = x[k];
  }
}

// contiguous pinned memory, coalesced: 1 KB per wave instruction, L in flight per lane
template <int L>
__global__ void __launch_bounds__(256) seq(const v4u* src, size_t n16, v4u* out) {
  const size_t i0 = ((size_t)blockIdx.x * 256 + threadIdx.x);
  const size_t stride = (size_t)gridDim.x * 256;
  v4u x[L];
#pragma unroll
  for (int k = 0; k < L; ++k) {
    const size_t i = i0 + k * stride;
    x[k] = *reinterpret_cast<gv4u>(reinterpret_cast<unsigned long long>(src + (i < n16 ? i : 0)));
  }
#pragma unroll
  for (int k = 0; k < L; ++k) {
    const size_t i = i0 + k * stride;
    if (i < n16) out[i] = x[k];
  }
}

template <typename F>
double time_ms(F launch, int reps = 10) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  launch();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r) launch();
  CHECK(hipEventRecord(b, 0));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

template <int Q, int L>
void run_gather(const char* name, const unsigned long long* ptrs, unsigned n, v4u* out) {
  constexpr unsigned FPW = L * 64 / Q;
  const unsigned waves = (n + FPW - 1) / FPW;
  const double ms = time_ms([&] { gather<Q, L><<<(waves + 3) / 4, 256>>>(ptrs, n, out); });
  printf("{\"pattern\": \"%s\", \"bytes_per_frame\": %d, \"loads_in_flight_per_lane\": %d, \"ms\": %.4f, "
         "\"mframes_s\": %.1f, \"gbs\": %.2f}\n",
         name, 16 * Q, L, ms, n / ms / 1e3, (double)n * 16 * Q / ms / 1e6);
}

// pool: 0 = hipHostMalloc, 1 = mmap + MADV_HUGEPAGE (transparent 2-MB pages) + hipHostRegister,
// 2 = hipHostMalloc with every frame in the first 64 MB of the pool (small translation footprint,
// but every buffer read ~70 times); 3 = each buffer once, in address order; 4 = each buffer once,
// frames bucketed by 64-MB region of the pool (random order within a region)
void run_pool(unsigned n, int mode) {
  const size_t buf = 2176, head = 128, bytes = (size_t)n * buf;
  unsigned char* pool = nullptr;
  if (mode == 1) {
    void* p = mmap(nullptr, bytes + (2u << 20), PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) { perror("mmap"); exit(1); }
    pool = reinterpret_cast<unsigned char*>((reinterpret_cast<uintptr_t>(p) + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1));
    madvise(pool, bytes, MADV_HUGEPAGE);
    for (size_t i = 0; i < bytes; i += 4096) pool[i] = (unsigned char)i;
    CHECK(hipHostRegister(pool, bytes, hipHostRegisterMapped));
  } else {
    CHECK(hipHostMalloc(reinterpret_cast<void**>(&pool), bytes, hipHostMallocMapped));
    for (size_t i = 0; i < bytes; i += 4096) pool[i] = (unsigned char)i;
  }
  std::vector<unsigned> perm(n);
  std::iota(perm.begin(), perm.end(), 0u);
  std::shuffle(perm.begin(), perm.end(), std::mt19937(7));
  const unsigned span = mode == 2 ? (unsigned)((64u << 20) / buf) : n;
  if (mode == 3) std::sort(perm.begin(), perm.end());
  if (mode == 4) {
    const unsigned per = (unsigned)((64u << 20) / buf);
    std::stable_sort(perm.begin(), perm.end(), [per](unsigned x, unsigned y) { return x / per < y / per; });
  }
  unsigned long long* hp = nullptr;
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&hp), (size_t)n * 8, hipHostMallocMapped));
  void* dpool = nullptr;
  CHECK(hipHostGetDevicePointer(&dpool, pool, 0));
  for (unsigned i = 0; i < n; ++i)
    hp[i] = reinterpret_cast<unsigned long long>(dpool) + (size_t)(perm[i] % span) * buf + head;
  unsigned long long* dptrs = nullptr;
  CHECK(hipMalloc(&dptrs, (size_t)n * 8));
  CHECK(hipMemcpy(dptrs, hp, (size_t)n * 8, hipMemcpyHostToDevice));
  v4u* out = nullptr;
  CHECK(hipMalloc(&out, (size_t)n * 256));
  const char* names[] = {"hipHostMalloc pool", "THP pool + hipHostRegister", "frames within 64 MB",
                         "address order", "bucketed by 64-MB region"};
  char name[128];
  snprintf(name, sizeof(name), "%s, 4 lanes/frame", names[mode]);
  run_gather<4, 16>(name, dptrs, n, out);
  snprintf(name, sizeof(name), "%s, 8 lanes/frame", names[mode]);
  run_gather<8, 16>(name, dptrs, n, out);
  if (mode == 0) {
    unsigned long long* dp = nullptr;
    CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dp), hp, 0));
    run_gather<4, 16>("hipHostMalloc pool, ptrs in host memory", dp, n, out);
    const size_t n16 = (size_t)n * 4;
    for (int blocks : {4096, 16384}) {
      const double ms = time_ms([&] { seq<8><<<blocks, 256>>>(reinterpret_cast<const v4u*>(dpool), n16, out); });
      printf("{\"pattern\": \"sequential pinned, %d blocks\", \"bytes\": %zu, \"ms\": %.4f, \"gbs\": %.2f}\n", blocks,
             n16 * 16, ms, n16 * 16 / ms / 1e6);
    }
    const double ms = time_ms([&] { CHECK(hipMemcpyAsync(out, pool, n16 * 16, hipMemcpyHostToDevice, 0)); });
    printf("{\"pattern\": \"hipMemcpyAsync H2D\", \"bytes\": %zu, \"ms\": %.4f, \"gbs\": %.2f}\n", n16 * 16, ms,
           n16 * 16 / ms / 1e6);
  }
  CHECK(hipFree(out));
  CHECK(hipFree(dptrs));
  CHECK(hipHostFree(hp));
  if (mode == 1) CHECK(hipHostUnregister(pool));
  else CHECK(hipHostFree(pool));
}

int main(int argc, char** argv) {
  const unsigned n = argc > 1 ? (unsigned)atoi(argv[1]) : (1u << 21);
  for (int mode = 0; mode < 5; ++mode) run_pool(n, mode);
  return 0;
}
