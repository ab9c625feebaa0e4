// Gather kernel of rtn_stage_gather (include/retina_stage.h) for gfx950: DPDK mbufs in a host
// mbuf pool the GPU maps (hipHostRegister) -> the compact split layout of retina_pc.h in HBM,
// with no host copy. The reference reads each header straight out of its mbuf at
// buf_addr + data_off + offset (Mbuf::get_data, core/src/memory/mbuf.rs:125-141) after rx_burst
// (core/src/lcore/rx_core.rs:57-73); here one wave pulls 256 mbufs' first 64 bytes (and bytes
// [64, 128) of those rtn_ext_needed names) across PCIe and writes them as head slots / ext rows.
//
// One wave per 256-frame chunk (RTN_CHUNK_FRAMES), four waves per block. Per wave:
//   1. lane l holds the data pointer and data_len of frames l, l+64, l+128, l+192 of the chunk
//      (coalesced reads of the pointer array); a pointer outside the registered pool is never
//      dereferenced: its frame gets data_len 0 and RTN_STATUS_BAD_MBUF;
//   2. head slots: 16 loads per lane, each covering 16 frames -- lane l reads quarter l%4 of frame
//      16k + l/4, so four lanes read one mbuf's 64 contiguous bytes (one 64-B PCIe read) -- all
//      issued before the first store, then stored as 1-KB coalesced runs;
//   3. rtn_ext_needed from the quarter-0 lane's bytes 12..15, its neighbour's bytes 16..19 and
//      data_len; a ballot gives the chunk's 256-bit need mask;
//   4. ext rows: the needing frames' pointers are ranked into a per-wave LDS list, then read 16
//      frames per load (again four lanes per mbuf) and stored at rows c*256 + rank.
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif

typedef unsigned int rtn_u32;
typedef unsigned long long rtn_u64;
typedef unsigned int rtn_v4u __attribute__((ext_vector_type(4)));
// host memory mapped for the device, read through the global address space
typedef const __attribute__((address_space(1))) rtn_v4u* rtn_gv4u;

struct rtn_stage_args {
  const rtn_u64* ptrs;           // [n] host virtual addresses of the frames' data (buf_addr + data_off)
  const unsigned short* dl_in;   // [n] Mbuf::data_len
  unsigned char* head;           // [ceil(n/256)*256][64] head slots (device)
  unsigned char* ext;            // [ceil(n/256)*256][64] ext rows, chunk c at rows [c*256, ...)
  rtn_u32* ext_chunk;            // [ceil(n/256)] = c * 256
  unsigned short* dlen;          // [n] data_len as the filter reads it (0 for a bad pointer)
  rtn_u32* status;               // RTN_STATUS_BAD_MBUF (8) by atomic OR
  rtn_u64 lo, hi;                // the registered pool: a pointer p is read iff lo <= p <= hi - 128
  rtn_u64 delta;                 // device address = host address + delta (mod 2^64)
  rtn_u32 n;
};

__device__ __forceinline__ rtn_u64 rtn_shfl64(rtn_u64 v, rtn_u32 src) {
  const rtn_u32 lo = __shfl((rtn_u32)v, (int)src), hi = __shfl((rtn_u32)(v >> 32), (int)src);
  return (rtn_u64)lo | ((rtn_u64)hi << 32);
}

// rtn_ext_needed (retina_pc.h) from the words holding bytes 12..15 and 16..19 of the frame.
__device__ __forceinline__ bool rtn_stage_need(rtn_u32 w3, rtn_u32 w4, rtn_u32 dl) {
  const rtn_u32 et = __builtin_amdgcn_perm(0u, w3, 0x0c0c0001u);  // bytes 12..13 big-endian
  const bool q = et == 0x8100u;
  const rtn_u32 inner = q ? __builtin_amdgcn_perm(0u, w4, 0x0c0c0001u) : et;  // bytes 16..17
  const rtn_u32 vihl = q ? (w4 >> 16) & 0xffu : (w3 >> 16) & 0xffu;           // byte 18 / 14
  const rtn_u32 l4 = (q ? 18u : 14u) + (inner == 0x86DDu ? 40u : ((vihl & 0xfu) << 2));
  const bool ip = inner == 0x0800u || inner == 0x86DDu;
  return ip && dl > 64u && l4 + 20u > 64u;
}

// bits 0, 4, 8, ..., 60 of x -> bits 0..15
__device__ __forceinline__ rtn_u32 rtn_every4(rtn_u64 x) {
  x &= 0x1111111111111111ull;
  x = (x | (x >> 3)) & 0x0303030303030303ull;
  x = (x | (x >> 6)) & 0x000F000F000F000Full;
  x = (x | (x >> 12)) & 0x000000FF000000FFull;
  return (rtn_u32)((x | (x >> 24)) & 0xFFFFull);
}

__device__ __forceinline__ void rtn_stage_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

extern "C" __global__ void __launch_bounds__(256) rtn_stage_gather_kernel(rtn_stage_args a) {
  const rtn_u32 lane = threadIdx.x & 63u, q4 = lane & 3u;
  const rtn_u32 c = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
  const rtn_u32 nch = (a.n + 255u) >> 8;
  __shared__ rtn_u64 rtn_list[4][256];  // per wave: data pointers of the chunk's needing frames
  rtn_u64* list = rtn_list[threadIdx.x >> 6];
  if (c >= nch) return;  // wave-uniform
  const rtn_u32 base = c << 8;
  const rtn_u64 lane_lt = lane == 0u ? 0ull : (~0ull >> (64u - lane));
  // 1. pointers and data_len of frames lane + 64 j: all eight loads in flight before any use
  rtn_u64 v[4];
  rtn_u32 dv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const rtn_u32 i = base + lane + 64u * j, ic = i < a.n ? i : a.n - 1u;  // no branch around the load
    v[j] = a.ptrs[ic];
    dv[j] = a.dl_in[ic];
  }
  rtn_u64 p[4];
  rtn_u32 d[4];
  bool bad = false;
  const rtn_u64 safe = a.lo + a.delta;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const rtn_u32 i = base + lane + 64u * j;
    const bool ok = i < a.n && v[j] >= a.lo && v[j] <= a.hi - 128u;
    bad = bad || (i < a.n && !ok);
    p[j] = ok ? v[j] + a.delta : safe;
    d[j] = ok ? dv[j] : 0u;
  }
  // 2. head slots: lane l of load k reads quarter l%4 of frame 16k + l/4 (global loads: a flat
  // load would also count against lgkmcnt, and every cross-lane shuffle's wait would then wait
  // for the PCIe round trip)
  rtn_u64 pf[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) pf[k] = rtn_shfl64(p[k >> 2], 16u * (k & 3) + (lane >> 2)) + 16u * q4;
  rtn_v4u x[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) x[k] = *reinterpret_cast<rtn_gv4u>(pf[k]);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const rtn_u32 i = base + lane + 64u * j;
    if (i < a.n) a.dlen[i] = (unsigned short)d[j];
  }
  rtn_u64 need[4] = {0ull, 0ull, 0ull, 0ull};  // wave-uniform need mask of the chunk's 256 frames
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const rtn_u32 f = 16u * k + (lane >> 2), i = base + f;
    if (i < a.n) *reinterpret_cast<rtn_v4u*>(a.head + (rtn_u64)i * 64u + 16u * q4) = x[k];
    // 3. the quarter-0 lane of each frame decides rtn_ext_needed
    const rtn_u32 w4 = __shfl_down(x[k].x, 1u);
    const rtn_u32 dl = __shfl(d[k >> 2], (int)(16u * (k & 3) + (lane >> 2)));
    const bool nd = q4 == 0u && i < a.n && rtn_stage_need(x[k].w, w4, dl);
    need[k >> 2] |= (rtn_u64)rtn_every4(__ballot(nd)) << (16u * (k & 3));
  }
  // 4. ext rows: rank the needing frames into the LDS list, then copy 16 frames per load
  rtn_u32 total = 0u;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const rtn_u64 m = need[j];
    if ((m >> lane) & 1ull) list[total + (rtn_u32)__popcll(m & lane_lt)] = p[j];
    total += (rtn_u32)__popcll(m);
  }
  rtn_stage_wave_sync();
  rtn_v4u y[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const rtn_u32 e = 16u * t + (lane >> 2);
    if (16u * t < total) {
      const rtn_u64 pe = e < total ? list[e] : safe;
      y[t] = *reinterpret_cast<rtn_gv4u>(pe + 64u + 16u * q4);
    }
  }
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const rtn_u32 e = 16u * t + (lane >> 2);
    if (16u * t < total && e < total)
      *reinterpret_cast<rtn_v4u*>(a.ext + (rtn_u64)(base + e) * 64u + 16u * q4) = y[t];
  }
  if (lane == 0u) a.ext_chunk[c] = base;
  if (__ballot(bad) != 0ull && lane == 0u) atomicOr(a.status, 8u);
}
