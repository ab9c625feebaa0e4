// Staging DPDK RX bursts into the compact split layout (include/retina_stage.h).
//
// The reference hands the packet filter one mbuf at a time and reads each header in place at
// buf_addr + data_off + offset (Mbuf::get_data, core/src/memory/mbuf.rs:125-141), right after
// rx_burst (core/src/lcore/rx_core.rs:57-73, 117-141). The batched path instead gathers many
// bursts into one slab the GPU reads with coalesced loads:
//   (a) rtn_stage_mbufs: host worker threads copy each mbuf's first 64 bytes into its head slot
//       and, for the frames rtn_ext_needed names, bytes [64, 128) into the next ext row;
//   (b) rtn_stage_gather: the gfx950 kernel of stage_kernel.hip reads the mbufs straight out of
//       a registered host pool over PCIe and writes the same layout in HBM.
#include "retina_pc.h"
#include "retina_stage.h"

#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../runtime/rtn_error.hpp"

namespace {
#include "stage_kernel_src.inc"  // kStageKernelSrc: csrc/kernels/stage_kernel.hip

int32_t fail(int32_t code, const std::string& msg) { return rtn::set_error(code, msg); }
int32_t hip_fail(const char* what, hipError_t e) {
  return fail(RTN_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
}
// Below this many frames a gather runs on the calling thread (waking workers costs more).
constexpr uint32_t kInlineFrames = 8192;
// Mbufs whose first line is requested ahead of the copy (their pointers are known in advance, the
// lines are scattered over the pool: each one is a DRAM miss the copy would otherwise wait for).
constexpr uint32_t kPrefetch = 16;
}  // namespace

struct rtn_stager {
  std::vector<std::thread> workers;
  std::mutex mu;
  std::condition_variable wake, done;
  uint64_t gen = 0;
  uint32_t pending = 0;
  bool stop = false;
  std::function<void(uint32_t)> job;
  std::vector<uint64_t> need;       // per-call need bitmap (bit i: frame i has an ext row)
  std::vector<uint32_t> chunk_rows; // per-call needing frames of each chunk
  std::vector<uint16_t> dl_max;     // per-slice largest data_len

  // Runs job(0..workers) on the workers and waits for all of them.
  void run_all() {
    std::unique_lock<std::mutex> lk(mu);
    pending = (uint32_t)workers.size();
    ++gen;
    wake.notify_all();
    done.wait(lk, [&] { return pending == 0; });
  }
  void worker(uint32_t k) {
    uint64_t seen = 0;
    for (;;) {
      std::function<void(uint32_t)> f;
      {
        std::unique_lock<std::mutex> lk(mu);
        wake.wait(lk, [&] { return stop || gen != seen; });
        if (stop) return;
        seen = gen;
        f = job;
      }
      f(k);
      std::lock_guard<std::mutex> lk(mu);
      if (--pending == 0) done.notify_all();
    }
  }
  ~rtn_stager() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    wake.notify_all();
    for (auto& t : workers) t.join();
  }
};

namespace {

// 64 bytes into a head slot or ext row. Streaming stores when the slab is 64-B aligned: a head
// slot or ext row is written whole and read next by the DMA engine, so the plain copy's
// read-for-ownership of the destination line is pure waste (cfg2, 14 threads: 608 -> 1047 Mpkt/s,
// profiles/r3a_stage_probe_*). Each worker fences its own streaming stores before it reports done.
template <bool NT>
inline void copy64(uint8_t* dst, const uint8_t* src) {
  if (NT) {
    const __m128i* s = reinterpret_cast<const __m128i*>(src);
    __m128i* d = reinterpret_cast<__m128i*>(dst);
    const __m128i a = _mm_loadu_si128(s), b = _mm_loadu_si128(s + 1), c = _mm_loadu_si128(s + 2),
                  e = _mm_loadu_si128(s + 3);
    _mm_stream_si128(d, a);
    _mm_stream_si128(d + 1, b);
    _mm_stream_si128(d + 2, c);
    _mm_stream_si128(d + 3, e);
  } else {
    memcpy(dst, src, 64);
  }
}

// Pass 1 over frames [f0, f1) (whole chunks): head slots, data_len, need bits, rows per chunk.
template <bool NT>
void stage_heads(const uint8_t* const* data, const uint16_t* dl, uint32_t f0, uint32_t f1,
                 const rtn_stage_slab_t& s, uint64_t* need, uint32_t* chunk_rows, uint16_t& dl_max) {
  uint16_t mx = 0;
  for (uint32_t c = f0 / RTN_CHUNK_FRAMES; c * RTN_CHUNK_FRAMES < f1; ++c) chunk_rows[c] = 0;
  for (uint32_t w = f0 / 64u; w * 64u < f1; ++w) need[w] = 0;
  for (uint32_t i = f0; i < f1; ++i) {
    if (i + kPrefetch < f1) __builtin_prefetch(data[i + kPrefetch]);
    const uint8_t* src = data[i];
    uint8_t* h = s.head + (uint64_t)i * 64u;
    copy64<NT>(h, src);
    const uint16_t d = dl[i];
    s.data_len[i] = d;
    mx = d > mx ? d : mx;
    if (rtn_ext_needed(src, d)) {
      need[i / 64u] |= 1ull << (i % 64u);
      ++chunk_rows[i / RTN_CHUNK_FRAMES];
    }
  }
  dl_max = mx;
  if (NT) _mm_sfence();
}

// Pass 2: ext rows of the needing frames of [f0, f1), from ext_chunk (already the prefix).
template <bool NT>
void stage_ext(const uint8_t* const* data, uint32_t f0, uint32_t f1, const rtn_stage_slab_t& s,
               const uint64_t* need) {
  for (uint32_t c = f0 / RTN_CHUNK_FRAMES; c * RTN_CHUNK_FRAMES < f1; ++c) {
    uint64_t row = s.ext_chunk[c];
    const uint32_t w0 = c * (RTN_CHUNK_FRAMES / 64u), w1 = std::min(w0 + RTN_CHUNK_FRAMES / 64u, (f1 + 63u) / 64u);
    for (uint32_t w = w0; w < w1; ++w) {
      uint64_t b = need[w];
      // the next word's needing frames, requested while this word's are copied
      if (w + 1u < w1) {
        uint64_t nb = need[w + 1u];
        while (nb) {
          __builtin_prefetch(data[(w + 1u) * 64u + (uint32_t)__builtin_ctzll(nb)] + 64);
          nb &= nb - 1u;
        }
      }
      while (b) {
        const uint32_t i = w * 64u + (uint32_t)__builtin_ctzll(b);
        copy64<NT>(s.ext + row * 64u, data[i] + 64);
        ++row;
        b &= b - 1u;
      }
    }
  }
  if (NT) _mm_sfence();
}

void stage_heads_any(bool nt, const uint8_t* const* data, const uint16_t* dl, uint32_t f0, uint32_t f1,
                     const rtn_stage_slab_t& s, uint64_t* need, uint32_t* chunk_rows, uint16_t& dl_max) {
  if (nt)
    stage_heads<true>(data, dl, f0, f1, s, need, chunk_rows, dl_max);
  else
    stage_heads<false>(data, dl, f0, f1, s, need, chunk_rows, dl_max);
}

void stage_ext_any(bool nt, const uint8_t* const* data, uint32_t f0, uint32_t f1, const rtn_stage_slab_t& s,
                   const uint64_t* need) {
  if (nt)
    stage_ext<true>(data, f0, f1, s, need);
  else
    stage_ext<false>(data, f0, f1, s, need);
}

}  // namespace

extern "C" {

int32_t rtn_stager_create(uint32_t threads, const int32_t* cpus, rtn_stager_t** out) {
  if (!out) return fail(RTN_EINVAL, "null argument");
  if (threads > 1024) return fail(RTN_EINVAL, "at most 1024 stager threads");
  try {
    auto st = std::make_unique<rtn_stager>();  // (a failed create joins the workers it started)
    rtn_stager* raw = st.get();
    for (uint32_t k = 0; k < threads; ++k) {
      st->workers.emplace_back([raw, k] { raw->worker(k); });
      if (cpus) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(cpus[k], &set);
        pthread_setaffinity_np(st->workers.back().native_handle(), sizeof(set), &set);
      }
    }
    *out = st.release();
    return RTN_OK;
  } catch (const std::exception& e) {
    return fail(RTN_EDEVICE, std::string("rtn_stager_create: ") + e.what());
  }
}

void rtn_stager_destroy(rtn_stager_t* st) { delete st; }

int32_t rtn_stage_mbufs(rtn_stager_t* st, const uint8_t* const* data, const uint16_t* data_len, uint32_t n,
                        const rtn_stage_slab_t* slab, uint32_t* rows, uint16_t* dl_max) {
  if (!st || !slab || !rows) return fail(RTN_EINVAL, "null argument");
  *rows = 0;
  if (dl_max) *dl_max = 0;
  if (n == 0) return RTN_OK;
  if (!data || !data_len || !slab->head || !slab->ext_chunk || !slab->data_len)
    return fail(RTN_EINVAL, "null argument");
  if (n > slab->cap) return fail(RTN_ERANGE, "more frames than the slab holds");
  if (n > RTN_MAX_FRAMES) return fail(RTN_EINVAL, "batch larger than RTN_MAX_FRAMES");
  const uint32_t nch = (n + RTN_CHUNK_FRAMES - 1u) / RTN_CHUNK_FRAMES;
  try {
    st->need.resize(((size_t)n + 63u) / 64u);
    st->chunk_rows.resize(nch);
  } catch (const std::exception& e) {
    return fail(RTN_ERANGE, std::string("rtn_stage_mbufs: ") + e.what());
  }
  const rtn_stage_slab_t s = *slab;
  uint64_t* need = st->need.data();
  uint32_t* crow = st->chunk_rows.data();
  // streaming stores need 16-B-aligned destinations; slabs from pinned allocators are page aligned
  const bool nt = (((uintptr_t)s.head | (uintptr_t)s.ext) & 63u) == 0;
  const uint32_t T = (n < kInlineFrames || st->workers.empty()) ? 1u
                     : std::min<uint32_t>((uint32_t)st->workers.size(), nch);
  st->dl_max.assign(T, 0);
  // slice t: chunks [nch * t / T, nch * (t + 1) / T)
  auto lo = [&](uint32_t t) { return std::min<uint64_t>((uint64_t)nch * t / T * RTN_CHUNK_FRAMES, n); };
  if (T == 1) {
    stage_heads_any(nt, data, data_len, 0, n, s, need, crow, st->dl_max[0]);
  } else {
    st->job = [&](uint32_t k) {
      if (k < T) stage_heads_any(nt, data, data_len, (uint32_t)lo(k), (uint32_t)lo(k + 1), s, need, crow, st->dl_max[k]);
    };
    st->run_all();
  }
  uint64_t r = 0;
  for (uint32_t c = 0; c < nch; ++c) {
    s.ext_chunk[c] = (uint32_t)r;
    r += crow[c];
  }
  uint16_t mx = 0;
  for (uint16_t v : st->dl_max) mx = v > mx ? v : mx;
  if (dl_max) *dl_max = mx;
  if (r > s.ext_cap) return fail(RTN_ERANGE, "the frames need more ext rows than the slab holds");
  if (r && !s.ext) return fail(RTN_EINVAL, "ext rows needed but slab->ext is null");
  if (r) {
    if (T == 1) {
      stage_ext_any(nt, data, 0, n, s, need);
    } else {
      st->job = [&](uint32_t k) {
        if (k < T) stage_ext_any(nt, data, (uint32_t)lo(k), (uint32_t)lo(k + 1), s, need);
      };
      st->run_all();
    }
  }
  *rows = (uint32_t)r;
  return RTN_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// (b) GPU pull from a registered mbuf pool

struct rtn_mbuf_pool {
  int device = 0;
  uint8_t* base = nullptr;
  size_t bytes = 0;
  uint64_t delta = 0;       // device address - host address
  bool registered = false;  // we registered it (else it was pinned already)
  hipModule_t module = nullptr;
  hipFunction_t fn = nullptr;
  uint32_t* status = nullptr;  // sticky status word of gathers without a status pointer
  hipEvent_t last = nullptr;   // recorded after each such gather
  hipStream_t own = nullptr;   // private stream of rtn_mbuf_pool_take_status
  ~rtn_mbuf_pool() {
    if (status) (void)hipFree(status);
    if (last) (void)hipEventDestroy(last);
    if (own) (void)hipStreamDestroy(own);
    if (module) (void)hipModuleUnload(module);
    if (registered) (void)hipHostUnregister(base);
  }
};

namespace {
struct StageArgs {  // must match struct rtn_stage_args in stage_kernel.hip
  const uint64_t* ptrs;
  const uint16_t* dl_in;
  uint8_t* head;
  uint8_t* ext;
  uint32_t* ext_chunk;
  uint16_t* dlen;
  uint32_t* status;
  uint64_t lo, hi;
  uint64_t delta;
  uint32_t n;
};
}  // namespace

extern "C" {

int32_t rtn_mbuf_pool_register(void* base, size_t bytes, int device, rtn_mbuf_pool_t** out) {
  if (!base || !out) return fail(RTN_EINVAL, "null argument");
  if (bytes < 128) return fail(RTN_EINVAL, "a pool holds at least 128 bytes");
  std::shared_ptr<std::vector<uint8_t>> code;
  int32_t rc = rtn::compile_hip(kStageKernelSrc, code);
  if (rc) return rc;
  auto pool = std::make_unique<rtn_mbuf_pool>();
  pool->device = device;
  pool->base = static_cast<uint8_t*>(base);
  pool->bytes = bytes;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return hip_fail("hipSetDevice", e);
  // memory pinned by its allocator (hipHostMalloc, a pinned torch tensor) is mapped as it is;
  // anything else is registered here and unregistered by rtn_mbuf_pool_destroy
  hipPointerAttribute_t attr;
  const bool pinned = hipPointerGetAttributes(&attr, base) == hipSuccess && attr.type == hipMemoryTypeHost;
  (void)hipGetLastError();
  if (!pinned) {
    e = hipHostRegister(base, bytes, hipHostRegisterMapped);
    if (e != hipSuccess) return hip_fail("hipHostRegister", e);
    pool->registered = true;
  }
  void* dptr = nullptr;
  e = hipHostGetDevicePointer(&dptr, base, 0);
  if (e != hipSuccess) return hip_fail("hipHostGetDevicePointer", e);
  pool->delta = reinterpret_cast<uint64_t>(dptr) - reinterpret_cast<uint64_t>(base);
  e = hipModuleLoadData(&pool->module, code->data());
  if (e != hipSuccess) return hip_fail("hipModuleLoadData", e);
  e = hipModuleGetFunction(&pool->fn, pool->module, "rtn_stage_gather_kernel");
  if (e != hipSuccess) return hip_fail("hipModuleGetFunction", e);
  e = hipMalloc(reinterpret_cast<void**>(&pool->status), 4);
  if (e == hipSuccess) e = hipMemset(pool->status, 0, 4);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&pool->last, hipEventDisableTiming);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&pool->own, hipStreamNonBlocking);
  if (e != hipSuccess) return hip_fail("rtn_mbuf_pool_register", e);
  *out = pool.release();
  return RTN_OK;
}

int32_t rtn_mbuf_pool_destroy(rtn_mbuf_pool_t* pool) {
  delete pool;
  return RTN_OK;
}

uint32_t rtn_stage_gather_ext_rows(uint32_t n) {
  return (uint32_t)(((uint64_t)n + RTN_CHUNK_FRAMES - 1u) / RTN_CHUNK_FRAMES * RTN_CHUNK_FRAMES);
}

int32_t rtn_stage_gather(rtn_mbuf_pool_t* pool, const uint64_t* data, const uint16_t* data_len, uint32_t n,
                         const rtn_stage_slab_t* slab, uint32_t* status, void* stream) {
  if (!pool || !slab) return fail(RTN_EINVAL, "null argument");
  if (n == 0) return RTN_OK;
  if (!data || !data_len || !slab->head || !slab->ext || !slab->ext_chunk || !slab->data_len)
    return fail(RTN_EINVAL, "null argument");
  if (n > RTN_MAX_FRAMES) return fail(RTN_EINVAL, "batch larger than RTN_MAX_FRAMES");
  if (n > slab->cap) return fail(RTN_ERANGE, "more frames than the slab holds");
  if (slab->ext_cap < rtn_stage_gather_ext_rows(n))
    return fail(RTN_ERANGE, "the gather layout needs rtn_stage_gather_ext_rows(n) ext rows");
  if (((reinterpret_cast<uintptr_t>(slab->head) | reinterpret_cast<uintptr_t>(slab->ext)) & 15u) != 0)
    return fail(RTN_EINVAL, "head and ext must be 16-byte aligned");
  StageArgs a;
  a.ptrs = data;
  a.dl_in = data_len;
  a.head = slab->head;
  a.ext = slab->ext;
  a.ext_chunk = slab->ext_chunk;
  a.dlen = slab->data_len;
  a.status = status ? status : pool->status;
  a.lo = reinterpret_cast<uint64_t>(pool->base);
  a.hi = a.lo + pool->bytes;
  a.delta = pool->delta;
  a.n = n;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  void* params[] = {&a};
  const uint32_t chunks = (n + RTN_CHUNK_FRAMES - 1u) / RTN_CHUNK_FRAMES;
  hipError_t e = hipSetDevice(pool->device);
  if (e == hipSuccess) e = hipModuleLaunchKernel(pool->fn, (chunks + 3u) / 4u, 1, 1, 256, 1, 1, 0, s, params, nullptr);
  if (e == hipSuccess && !status) e = hipEventRecord(pool->last, s);
  return e == hipSuccess ? RTN_OK : hip_fail("rtn_stage_gather", e);
}

int32_t rtn_mbuf_pool_take_status(rtn_mbuf_pool_t* pool, uint32_t* status) {
  if (!pool || !status) return fail(RTN_EINVAL, "null argument");
  hipError_t e = hipSetDevice(pool->device);
  if (e == hipSuccess) e = hipEventSynchronize(pool->last);
  if (e == hipSuccess) e = hipMemcpyAsync(status, pool->status, 4, hipMemcpyDeviceToHost, pool->own);
  if (e == hipSuccess) e = hipMemsetAsync(pool->status, 0, 4, pool->own);
  if (e == hipSuccess) e = hipStreamSynchronize(pool->own);
  return e == hipSuccess ? RTN_OK : hip_fail("rtn_mbuf_pool_take_status", e);
}

}  // extern "C"
