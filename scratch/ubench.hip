// Throwaway microbenchmark: how fast can gfx950 stream 64-B packet slots through
// (a) per-lane direct dwordx4 loads, (b) coalesced loads staged in LDS (padded),
// (c) a pure coalesced read (ceiling). Not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ void gen64(uint8_t* slab, uint16_t* dlen, uint32_t n, uint64_t seed) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t r0 = splitmix64(seed ^ (uint64_t)i * 8 + 0), r1 = splitmix64(seed ^ ((uint64_t)i * 8 + 1));
  uint64_t r2 = splitmix64(seed ^ ((uint64_t)i * 8 + 2)), r3 = splitmix64(seed ^ ((uint64_t)i * 8 + 3));
  uint8_t b[64];
  for (int k = 0; k < 64; ++k) b[k] = 0;
  for (int k = 0; k < 6; ++k) { b[k] = (uint8_t)(r0 >> (8 * k)); b[6 + k] = (uint8_t)(r1 >> (8 * k)); }
  b[12] = 0x08; b[13] = 0x00;
  b[14] = 0x45; b[15] = 0; b[16] = 0; b[17] = 50; b[22] = 64; b[23] = 6;
  for (int k = 0; k < 4; ++k) { b[26 + k] = (uint8_t)(r2 >> (8 * k)); b[30 + k] = (uint8_t)(r2 >> (32 + 8 * k)); }
  uint16_t sport = (uint16_t)r3, dport;
  if (((r3 >> 16) & 3) == 0) dport = 80; else { dport = (uint16_t)(r3 >> 24); if (dport == 80) dport = 81; }
  b[34] = sport >> 8; b[35] = sport & 0xff; b[36] = dport >> 8; b[37] = dport & 0xff;
  for (int k = 0; k < 4; ++k) { b[38 + k] = (uint8_t)(r1 >> (8 * k)); b[42 + k] = (uint8_t)(r0 >> (8 * k + 16)); }
  b[46] = 0x50; b[47] = (uint8_t)(r3 >> 40);
  for (int k = 0; k < 64; ++k) slab[(uint64_t)i * 64 + k] = b[k];
  dlen[i] = 64;
}

struct Rec { uint32_t idx, src, dst; uint16_t sp, dp; uint32_t seq, ack; uint16_t off, len; uint8_t proto, flags, ver, pad; };

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// (c) pure read ceiling: every lane reads 16 B per instruction, fully coalesced.
__global__ void __launch_bounds__(256) read_ceiling(const uint4* __restrict__ p, uint64_t n16, uint32_t* out) {
  uint32_t acc = 0;
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += stride) {
    uint4 v = p[i];
    acc ^= v.x + v.y + v.z + v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// (a) per-lane direct loads of the lane's own 64-B slot (4 x dwordx4), fixed-offset parse.
__global__ void __launch_bounds__(256) pc_direct(const uint4* __restrict__ slab, const uint16_t* __restrict__ dlen,
                                                  uint64_t* __restrict__ pc_bm, Rec* __restrict__ recs, uint32_t n) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave_g = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
  const uint32_t nw = (n + 63) / 64;
  for (uint32_t w = wave_g; w < nw; w += nwaves) {
    uint32_t i = w * 64 + lane;
    bool valid = i < n;
    uint4 q0 = {0,0,0,0}, q1 = q0, q2 = q0; uint16_t dl = 0;
    if (valid) { q0 = slab[(uint64_t)i * 4]; q1 = slab[(uint64_t)i * 4 + 1]; q2 = slab[(uint64_t)i * 4 + 2]; dl = dlen[i]; }
    (void)q0;
    // bytes: 12..13 ethertype in q0.w low half; fixed IHL=5 offsets for this probe
    uint32_t et = bswap32(q0.w) >> 16;
    uint32_t proto = (q1.z >> 8) & 0xff;           // byte 23
    uint32_t dport = bswap32(q2.y) & 0xffff;       // bytes 36..37
    bool pc = valid && dl >= 54 && et == 0x0800 && proto == 6 && dport == 80;
    uint64_t m = __ballot(pc);
    if (lane == 0) pc_bm[w] = m;
    if (pc) {
      uint32_t rank = __popcll(m & ((1ull << lane) - 1));
      Rec r;
      r.idx = i; r.src = bswap32((q1.w >> 16) | (q2.x << 16)); r.dst = bswap32((q2.x >> 16) | (q2.y << 16));
      r.sp = bswap32(q2.y) >> 16; r.dp = dport; r.seq = 0; r.ack = 0; r.off = 54; r.len = 10; r.proto = 6; r.flags = 0; r.ver = 4; r.pad = 0;
      recs[(uint64_t)w * 64 + rank] = r;
    }
  }
}

// (b) coalesced 4 KiB per wave into LDS (stride 68 B per packet: conflict-free dword reads), per-lane parse from LDS.
#define PST 68
__global__ void __launch_bounds__(256) pc_lds(const uint4* __restrict__ slab, const uint16_t* __restrict__ dlen,
                                               uint64_t* __restrict__ pc_bm, Rec* __restrict__ recs, uint32_t n) {
  __shared__ uint32_t lds[4][64 * PST / 4];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t* buf = lds[wv];
  const uint32_t wave_g = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
  const uint32_t nw = n / 64;  // full waves only in this probe
  for (uint32_t w = wave_g; w < nw; w += nwaves) {
    const uint4* src = slab + (uint64_t)w * 256;
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = src[k * 64 + lane];
    uint16_t dl = dlen[w * 64 + lane];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint32_t c = k * 64 + lane;           // 16-B chunk index in the 4 KiB tile
      uint32_t p = c >> 2, q = c & 3;
      uint32_t* d = buf + (p * PST + q * 16) / 4;
      d[0] = v[k].x; d[1] = v[k].y; d[2] = v[k].z; d[3] = v[k].w;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const uint8_t* pk = reinterpret_cast<const uint8_t*>(buf) + lane * PST;
    auto rd16 = [&](uint32_t o) -> uint32_t { return ((uint32_t)pk[o] << 8) | pk[o + 1]; };
    auto rd32 = [&](uint32_t o) -> uint32_t { return (rd16(o) << 16) | rd16(o + 2); };
    uint32_t et = rd16(12);
    uint32_t l3 = 14;
    uint32_t ihl = (pk[l3] & 0xf) * 4;
    uint32_t proto = pk[l3 + 9];
    uint32_t l4 = l3 + ihl;
    bool ok = dl >= 14 && et == 0x0800 && l3 + 20 <= dl && proto == 6 && l4 < dl && l4 + 20 <= dl;
    uint32_t dport = ok ? rd16(l4 + 2) : 0;
    bool pc = ok && dport == 80;
    uint64_t m = __ballot(pc);
    if (lane == 0) pc_bm[w] = m;
    if (pc) {
      uint32_t rank = __popcll(m & ((1ull << lane) - 1));
      Rec r;
      uint32_t thl = (pk[l4 + 12] & 0xf0) >> 2;
      uint32_t tot = rd16(l3 + 2);
      r.idx = w * 64 + lane; r.src = rd32(l3 + 12); r.dst = rd32(l3 + 16);
      r.sp = rd16(l4); r.dp = dport; r.seq = rd32(l4 + 4); r.ack = rd32(l4 + 8);
      r.off = l4 + thl; r.len = tot - (ihl + thl); r.proto = 6; r.flags = pk[l4 + 13]; r.ver = 4; r.pad = 0;
      recs[(uint64_t)w * 64 + rank] = r;
    }
    __builtin_amdgcn_wave_barrier();
  }
}

int main(int argc, char** argv) {
  uint32_t n = 1u << 25;
  int iters = 20;
  uint8_t* slab; uint16_t* dlen; uint64_t* bm; Rec* recs; uint32_t* scratch;
  CHECK(hipMalloc(&slab, (size_t)n * 64));
  CHECK(hipMalloc(&dlen, (size_t)n * 2));
  CHECK(hipMalloc(&bm, (size_t)(n / 64) * 8));
  CHECK(hipMalloc(&recs, (size_t)n * sizeof(Rec)));
  CHECK(hipMalloc(&scratch, 64));
  gen64<<<(n + 255) / 256, 256>>>(slab, dlen, n, 0x5EED0002ull);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch, double bytes_alg) {
    for (int w = 0; w < 3; ++w) launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    for (int it = 0; it < iters; ++it) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
    double s = ms / 1e3 / iters;
    printf("%-28s %8.3f ms  %9.1f Mpkt/s  %7.1f GB/s (alg)\n", name, s * 1e3, n / s / 1e6, bytes_alg / s / 1e9);
  };
  int cus = 256;
  for (int bpc : {4, 8, 16}) {
    int grid = cus * bpc;
    char nm[64];
    snprintf(nm, sizeof nm, "read_ceiling g=%d", grid);
    timeit(nm, [&] { read_ceiling<<<grid, 256>>>((const uint4*)slab, (uint64_t)n * 4, scratch); }, (double)n * 64);
    snprintf(nm, sizeof nm, "pc_direct g=%d", grid);
    timeit(nm, [&] { pc_direct<<<grid, 256>>>((const uint4*)slab, dlen, bm, recs, n); }, (double)n * 66);
    snprintf(nm, sizeof nm, "pc_lds g=%d", grid);
    timeit(nm, [&] { pc_lds<<<grid, 256>>>((const uint4*)slab, dlen, bm, recs, n); }, (double)n * 66);
  }
  // sanity: count accepted
  std::vector<uint64_t> h(n / 64);
  CHECK(hipMemcpy(h.data(), bm, h.size() * 8, hipMemcpyDeviceToHost));
  uint64_t c = 0; for (auto x : h) c += __builtin_popcountll(x);
  printf("accepted %llu of %u (%.4f)\n", (unsigned long long)c, n, (double)c / n);
  return 0;
}
