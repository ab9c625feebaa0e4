// Offline ingest: libpcap / pcapng capture -> slot slab + data_len, the host side of the batched
// packet stage (include/retina_ingest.h). Reference behaviour: core/src/runtime/offline.rs:64-82
// (read every frame, skip frames whose original length exceeds the mtu, mbuf data = captured
// bytes) and core/src/memory/mbuf.rs:56-76 (Mbuf::from_bytes). The file is memory-mapped and
// walked once; packing is a bounded memcpy per frame.
#include "retina_ingest.h"

#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../runtime/rtn_error.hpp"
#include "retina_pc.h"
#include "retina_stage.h"

namespace rtn_gpu_walk {
struct State;
void destroy(State* g);
}  // namespace rtn_gpu_walk

namespace {

enum class Fmt { Pcap, Pcapng };

inline uint32_t rd32(const uint8_t* p, bool swap) {
  uint32_t v;
  memcpy(&v, p, 4);
  return swap ? __builtin_bswap32(v) : v;
}
inline uint16_t rd16(const uint8_t* p, bool swap) {
  uint16_t v;
  memcpy(&v, p, 2);
  return swap ? __builtin_bswap16(v) : v;
}

}  // namespace

struct rtn_pcap {
  const uint8_t* base = nullptr;
  size_t size = 0;
  size_t off = 0;       // next record / block
  size_t first = 0;     // offset of the first record / block (rewind)
  Fmt fmt = Fmt::Pcap;
  bool swap = false;    // file byte order differs from the host's
  uint32_t mtu = 0;
  rtn_pcap_stats_t st{};
  size_t populated = 0;  // page tables mapped up to here (prefault)
  size_t prefetched = 0; // cache lines requested up to here (prefetch_ahead)
  rtn_gpu_walk::State* gpu = nullptr;  // rtn_pcap_next_batch_gpu's device state
};

namespace {

// Map the page tables a batch will read in one call (MADV_POPULATE_READ, Linux 5.14+) instead of
// taking a fault per 64 KB inside the packing loop. Best effort: older kernels fault as before.
void prefault(rtn_pcap* p, size_t off, size_t bytes) {
#ifdef MADV_POPULATE_READ
  const size_t page = 4096, end = (p->size + page - 1) & ~(page - 1);
  const size_t a = (off > p->populated ? off : p->populated) & ~(page - 1);
  size_t b = (off + bytes + page - 1) & ~(page - 1);
  if (b > end) b = end;
  if (b <= a) return;
  (void)madvise(const_cast<uint8_t*>(p->base) + a, b - a, MADV_POPULATE_READ);
  p->populated = b;
#else
  (void)p;
  (void)off;
  (void)bytes;
#endif
}

// The walk is a chain of dependent loads (each record header's offset comes from the previous
// one's length), one cache miss per record on captures of full-size frames. Records are
// contiguous, so the lines a few KB ahead of the walk will be read whatever their record
// boundaries: requesting them early turns the chain of misses into a stream (IMIX capture,
// 2^21 frames: 16.4 -> 27 Mpkt/s packed into the compact split layout, this container).
// Captures of small frames are read line after line anyway; the prefetch runs once the mean
// frame seen so far is long enough to skip lines.
constexpr size_t kPrefetchAhead = 4096;
constexpr uint64_t kPrefetchMinMean = 192;
inline void prefetch_ahead(rtn_pcap* p) {
  if (p->st.packed < 64 || p->st.bytes < kPrefetchMinMean * p->st.packed) return;
  const size_t end = p->off + kPrefetchAhead < p->size ? p->off + kPrefetchAhead : p->size;
  if (p->prefetched < p->off) p->prefetched = p->off & ~size_t(63);
  for (; p->prefetched < end; p->prefetched += 64) __builtin_prefetch(p->base + p->prefetched);
}

// Next frame of the capture: captured bytes + original length. Returns false at end of file
// (a truncated trailing record ends the file, as libpcap does).
bool next_frame(rtn_pcap* p, const uint8_t*& data, uint32_t& caplen, uint32_t& origlen) {
  if (p->fmt == Fmt::Pcap) {
    if (p->off + 16 > p->size) return false;
    const uint8_t* h = p->base + p->off;
    caplen = rd32(h + 8, p->swap);
    origlen = rd32(h + 12, p->swap);
    if (p->off + 16 + (size_t)caplen > p->size) return false;
    data = h + 16;
    p->off += 16 + (size_t)caplen;
    return true;
  }
  // pcapng: walk blocks until an enhanced (6) or simple (3) packet block
  while (p->off + 12 <= p->size) {
    const uint8_t* b = p->base + p->off;
    uint32_t type = rd32(b, p->swap);
    if (type == 0x0A0D0D0Au) {  // section header: its byte-order magic sets the section's order
      uint32_t bom;
      memcpy(&bom, b + 8, 4);
      p->swap = bom != 0x1A2B3C4Du;
    }
    uint32_t blen = rd32(b + 4, p->swap);
    if (blen < 12 || p->off + blen > p->size) return false;
    p->off += blen;
    if (type == 6 && blen >= 32) {
      caplen = rd32(b + 20, p->swap);
      origlen = rd32(b + 24, p->swap);
      if (28 + (size_t)caplen > blen) return false;
      data = b + 28;
      return true;
    }
    if (type == 3 && blen >= 16) {
      origlen = rd32(b + 8, p->swap);
      caplen = origlen < blen - 16 ? origlen : blen - 16;
      data = b + 12;
      return true;
    }
  }
  return false;
}

}  // namespace

extern "C" {

int32_t rtn_pcap_open(const char* path, uint32_t mtu, rtn_pcap_t** out) {
  if (!path || !out) return rtn::set_error(RTN_EINVAL, "null argument");
  int fd = open(path, O_RDONLY);
  if (fd < 0) return rtn::set_error(RTN_EINVAL, std::string("cannot open ") + path);
  struct stat sb;
  if (fstat(fd, &sb) != 0 || sb.st_size < 12) {
    close(fd);
    return rtn::set_error(RTN_EINVAL, std::string("not a capture file: ") + path);
  }
  void* m = mmap(nullptr, (size_t)sb.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
  close(fd);
  if (m == MAP_FAILED) return rtn::set_error(RTN_EINVAL, std::string("mmap failed: ") + path);
  auto* p = new rtn_pcap();
  p->base = static_cast<const uint8_t*>(m);
  p->size = (size_t)sb.st_size;
  p->mtu = mtu;
  uint32_t magic;
  memcpy(&magic, p->base, 4);
  if (magic == 0xA1B2C3D4u || magic == 0xA1B23C4Du || magic == 0xD4C3B2A1u || magic == 0x4D3CB2A1u) {
    if (p->size < 24) {
      rtn_pcap_close(p);
      return rtn::set_error(RTN_EINVAL, "truncated pcap header");
    }
    p->fmt = Fmt::Pcap;
    p->swap = magic == 0xD4C3B2A1u || magic == 0x4D3CB2A1u;
    p->first = 24;
  } else if (magic == 0x0A0D0D0Au) {
    p->fmt = Fmt::Pcapng;
    p->first = 0;
  } else {
    rtn_pcap_close(p);
    return rtn::set_error(RTN_EINVAL, std::string("unknown capture format: ") + path);
  }
  p->off = p->first;
  *out = p;
  return RTN_OK;
}

int32_t rtn_pcap_next_batch(rtn_pcap_t* p, uint8_t* slab, uint64_t stride, uint16_t* data_len, uint32_t cap,
                            uint32_t* n) {
  if (!p || !slab || !data_len || !n) return rtn::set_error(RTN_EINVAL, "null argument");
  if (stride == 0) return rtn::set_error(RTN_EINVAL, "stride must be positive");
  // about the bytes this batch reads: its frames at the capture's mean size so far, plus headers
  prefault(p, p->off, (size_t)cap * (p->st.packed ? p->st.bytes / p->st.packed + 32u : 128u) + (1u << 20));
  uint32_t k = 0;
  while (k < cap) {
    const uint8_t* data;
    uint32_t caplen, origlen;
    const size_t at = p->off;
    prefetch_ahead(p);
    if (!next_frame(p, data, caplen, origlen)) break;
    p->st.frames++;
    if (origlen > p->mtu) {  // offline.rs:68-70
      p->st.skipped_mtu++;
      continue;
    }
    if (caplen > 0xFFFFu) {  // Mbuf::data_len is a u16; the reference's from_bytes bails
      p->off = at;
      p->st.frames--;
      *n = k;
      return rtn::set_error(RTN_ERANGE, "captured frame longer than 65535 bytes");
    }
    memcpy(slab + (uint64_t)k * stride, data, caplen < stride ? caplen : stride);
    data_len[k] = (uint16_t)caplen;
    p->st.packed++;
    p->st.bytes += caplen;
    ++k;
  }
  *n = k;
  return RTN_OK;
}

int32_t rtn_pcap_next_batch_split(rtn_pcap_t* p, uint8_t* head, uint8_t* ext, uint32_t ext_cap, uint32_t* ext_chunk,
                                  uint16_t* data_len, uint32_t cap, uint32_t* n, uint32_t* rows) {
  if (!p || !head || !ext || !ext_chunk || !data_len || !n || !rows) return rtn::set_error(RTN_EINVAL, "null argument");
  prefault(p, p->off, (size_t)cap * (p->st.packed ? p->st.bytes / p->st.packed + 32u : 128u) + (1u << 20));
  uint32_t k = 0, r = 0;
  while (k < cap) {
    const uint8_t* data;
    uint32_t caplen, origlen;
    const size_t at = p->off;
    prefetch_ahead(p);
    if (!next_frame(p, data, caplen, origlen)) break;
    p->st.frames++;
    if (origlen > p->mtu) {  // offline.rs:68-70
      p->st.skipped_mtu++;
      continue;
    }
    if (caplen > 0xFFFFu) {
      p->off = at;
      p->st.frames--;
      *n = k;
      *rows = r;
      return rtn::set_error(RTN_ERANGE, "captured frame longer than 65535 bytes");
    }
    uint8_t* h = head + (uint64_t)k * 64u;
    memcpy(h, data, caplen < 64u ? caplen : 64u);
    const bool need = rtn_ext_needed(h, (uint16_t)caplen);
    if (need && r == ext_cap) {  // no row left: end the batch before this frame
      p->off = at;
      p->st.frames--;
      if (k == 0) {  // an empty batch always means end of file: say why this one is empty
        *n = 0;
        *rows = 0;
        return rtn::set_error(RTN_ERANGE, "no ext row free for the next frame (ext_cap too small)");
      }
      break;
    }
    if (k % RTN_CHUNK_FRAMES == 0) ext_chunk[k / RTN_CHUNK_FRAMES] = r;
    if (need) {
      const uint32_t m = caplen - 64u < 64u ? caplen - 64u : 64u;
      memcpy(ext + (uint64_t)r * 64u, data + 64, m);
      if (m < 64u) memset(ext + (uint64_t)r * 64u + m, 0, 64u - m);
      ++r;
    }
    data_len[k] = (uint16_t)caplen;
    p->st.packed++;
    p->st.bytes += caplen;
    ++k;
  }
  *n = k;
  *rows = r;
  return RTN_OK;
}

int32_t rtn_pcap_stats(const rtn_pcap_t* p, rtn_pcap_stats_t* st) {
  if (!p || !st) return rtn::set_error(RTN_EINVAL, "null argument");
  *st = p->st;
  return RTN_OK;
}

int32_t rtn_pcap_rewind(rtn_pcap_t* p) {
  if (!p) return rtn::set_error(RTN_EINVAL, "null argument");
  p->off = p->first;
  p->prefetched = 0;
  if (p->fmt == Fmt::Pcapng) p->swap = false;
  return RTN_OK;
}

void rtn_pcap_close(rtn_pcap_t* p) {
  if (!p) return;
  rtn_gpu_walk::destroy(p->gpu);
  if (p->base) munmap(const_cast<uint8_t*>(p->base), p->size);
  delete p;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// rtn_pcap_next_batch_gpu: the capture walk on the GPU (csrc/kernels/capwalk_kernel.hip). A window
// of the file, starting at a record, is copied to HBM as it is (the window's pages of the file
// mapping are registered with HIP and the copy engine reads them; if registration fails, worker
// threads copy them into pinned memory first); the kernels find the window's record
// chain, apply the offline runtime's rules and pack the kept frames into the gather layout of
// rtn_stage_gather; the window stays resident, so a batch cut short by `cap` continues from it.
namespace rtn_gpu_walk {
#include "capwalk_kernel_src.inc"  // kCapwalkKernelSrc

constexpr uint64_t kSeg = 4096;  // RTN_CAP_SEG
constexpr uint32_t kCand = 8;    // RTN_CAP_C
constexpr uint64_t kStop = 1ull << 63, kEof = 1ull << 61, kErr = 1ull << 60, kDead = 1ull << 59;
constexpr uint64_t kOffMask = 0xFFFFFFFFFFFFull;
constexpr uint64_t kPad = 256;  // readable bytes past a window (unaligned word reads, ext rows)

struct CapArgs {  // rtn_cap_args
  const uint8_t* win;
  uint64_t bytes;
  uint32_t nseg, fmt, swap, mtu, at_eof, levels, k, pad0;
  uint64_t* cand;
  uint32_t* ncand;
  uint64_t* nexit;
  uint32_t* ncnt;
  uint32_t* jump;
  uint32_t* path;
  uint32_t* pre;
  uint32_t* red;
  uint32_t* tgt;
  uint32_t cap, pad1;
  uint64_t* ptrs;
  uint16_t* dlen;
  uint64_t* cut;
};
struct PackArgs {  // rtn_cap_pack_args
  const uint64_t* ptrs;
  const uint16_t* dl;
  uint8_t* head;
  uint8_t* ext;
  uint32_t* ext_chunk;
  uint16_t* dlen;
  uint32_t n;
};
struct Res {  // device result block, copied back once per window
  uint64_t cut[4];
  uint32_t red[4];
  uint32_t tgt[2];
};

struct State {
  int device = -1;
  uint64_t window = 64ull << 20;
  hipModule_t module = nullptr;
  hipFunction_t cand = nullptr, nodes = nullptr, jump = nullptr, lift = nullptr, scan = nullptr, emit = nullptr,
                pack = nullptr;
  // two device buffers of 2 * half + kPad bytes: a window sits at [half, 2 * half) of one, the
  // next window's bytes are prefetched into the other's second half while the batches of the
  // current one run, and the current window's unread tail is moved in front of them on the switch
  uint8_t* d_buf[2] = {nullptr, nullptr};
  uint64_t half = 0;
  int cur = 0;
  uint8_t* win_ptr = nullptr;  // the resident window's first byte
  uint8_t* h_stage = nullptr;  // pinned
  uint64_t h_cap = 0;
  // the window's pages of the file mapping, registered with HIP so the copy engine reads them
  // directly (no host copy); -1: registration failed once (or RTN_GPU_WALK_STAGED is set), so
  // windows go through h_stage
  void* reg = nullptr;
  int reg_mode = 0;
  // the prefetch of file bytes [pf_off, pf_off + pf_len) into d_buf[1 - cur] + half, on cs;
  // pf_reg: its registered pages (the first partial page is read through reg)
  hipStream_t cs = nullptr;
  hipEvent_t pf_done = nullptr, s_ready = nullptr;
  bool pf_valid = false;
  uint64_t pf_off = 0, pf_len = 0;
  void* pf_reg = nullptr;
  // the pages of the window after the prefetched one, registered ahead on a helper thread
  // (registration takes ~1.6 ms per 256 MiB of host time): [ahead_lo, ahead_hi), ok if registered
  std::thread ahead;
  uintptr_t ahead_lo = 0, ahead_hi = 0;
  bool ahead_ok = false;
  uint8_t* d_seg = nullptr;  // per-segment / per-node arrays for seg_cap segments
  uint32_t seg_cap = 0;
  Res* d_res = nullptr;
  Res* h_res = nullptr;
  uint64_t* d_ptrs = nullptr;
  uint16_t* d_dl = nullptr;
  uint32_t list_cap = 0;
  // the resident window: file bytes [win_off, win_off + win_len) at win_ptr
  size_t win_off = 0, win_len = 0;
  bool win_valid = false;
  uint64_t last_batch = 0;  // file bytes the last batch consumed
  double bpf = 0;           // ... per frame it packed
  hipEvent_t packed = nullptr;  // after the last batch's packing (it reads the window and frame list)
  hipEvent_t copied = nullptr;  // after the last window copy (it reads reg / h_stage)
};

// Waits for an outstanding prefetch and forgets it.
// Joins the helper and releases the pages it registered.
void drop_ahead(State* g) {
  if (g->ahead.joinable()) g->ahead.join();
  if (g->ahead_ok) (void)hipHostUnregister(reinterpret_cast<void*>(g->ahead_lo));
  g->ahead_ok = false;
  g->ahead_lo = g->ahead_hi = 0;
}

void drop_prefetch(State* g) {
  drop_ahead(g);
  if (!g->pf_valid) return;
  (void)hipEventSynchronize(g->pf_done);
  if (g->pf_reg) (void)hipHostUnregister(g->pf_reg);
  g->pf_reg = nullptr;
  g->pf_valid = false;
}

void destroy(State* g) {
  if (!g) return;
  if (g->device >= 0) (void)hipSetDevice(g->device);
  drop_prefetch(g);
  if (g->reg) {
    (void)hipEventSynchronize(g->copied);  // the last window copy may still read the pages
    (void)hipHostUnregister(g->reg);
  }
  for (uint8_t* b : g->d_buf)
    if (b) (void)hipFree(b);
  if (g->cs) (void)hipStreamDestroy(g->cs);
  if (g->pf_done) (void)hipEventDestroy(g->pf_done);
  if (g->s_ready) (void)hipEventDestroy(g->s_ready);
  if (g->h_stage) (void)hipHostFree(g->h_stage);
  if (g->d_seg) (void)hipFree(g->d_seg);
  if (g->d_res) (void)hipFree(g->d_res);
  if (g->h_res) (void)hipHostFree(g->h_res);
  if (g->d_ptrs) (void)hipFree(g->d_ptrs);
  if (g->d_dl) (void)hipFree(g->d_dl);
  if (g->packed) (void)hipEventDestroy(g->packed);
  if (g->copied) (void)hipEventDestroy(g->copied);
  if (g->module) (void)hipModuleUnload(g->module);
  delete g;
}

int32_t hip_fail(const char* what, hipError_t e) {
  return rtn::set_error(RTN_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

int32_t init(State* g, int device) {
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return hip_fail("hipSetDevice", e);
  std::shared_ptr<std::vector<uint8_t>> code;
  int32_t rc = rtn::compile_hip(kCapwalkKernelSrc, code);
  if (rc) return rc;
  e = hipModuleLoadData(&g->module, code->data());
  if (e != hipSuccess) return hip_fail("hipModuleLoadData", e);
  const char* names[] = {"rtn_cap_cand", "rtn_cap_nodes", "rtn_cap_jump", "rtn_cap_lift", "rtn_cap_scan", "rtn_cap_emit",
                         "rtn_cap_pack"};
  hipFunction_t* fns[] = {&g->cand, &g->nodes, &g->jump, &g->lift, &g->scan, &g->emit, &g->pack};
  for (int k = 0; k < 7; ++k) {
    e = hipModuleGetFunction(fns[k], g->module, names[k]);
    if (e != hipSuccess) return hip_fail("hipModuleGetFunction", e);
  }
  e = hipEventCreateWithFlags(&g->packed, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&g->copied, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventRecord(g->copied, nullptr);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&g->pf_done, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&g->s_ready, hipEventDisableTiming);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&g->cs, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&g->d_res), sizeof(Res));
  if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&g->h_res), sizeof(Res), hipHostMallocDefault);
  if (e != hipSuccess) return hip_fail("rtn_pcap_next_batch_gpu: result block", e);
  const char* v = getenv("RTN_GPU_WALK_STAGED");  // diagnostics: the staged copy, for comparison
  g->reg_mode = v && *v && *v != '0' ? -1 : 1;
  g->device = device;
  return RTN_OK;
}

// Pointer-jumping levels for nseg segments: the chain has at most nseg nodes.
uint32_t levels(uint32_t nseg) {
  uint32_t k = 1;
  while ((1ull << k) < (uint64_t)nseg + 1) ++k;
  return k;
}
// The per-segment arrays in one allocation, laid out by carve().
size_t seg_bytes(uint32_t nseg) {
  const size_t nodes = (size_t)nseg * kCand;
  return nodes * 8 + (size_t)nseg * 4 + nodes * 8 + nodes * 12 + (levels(nseg) + 1) * nodes * 4 + (size_t)nseg * 4 +
         (size_t)nseg * 8 + 64;
}
void carve(uint8_t* q, uint32_t nseg_cap, CapArgs& a) {
  const size_t nodes = (size_t)nseg_cap * kCand;
  a.cand = reinterpret_cast<uint64_t*>(q);
  q += nodes * 8;
  a.nexit = reinterpret_cast<uint64_t*>(q);
  q += nodes * 8;
  a.ncand = reinterpret_cast<uint32_t*>(q);
  q += (size_t)nseg_cap * 4;
  a.ncnt = reinterpret_cast<uint32_t*>(q);
  q += nodes * 12;
  a.path = reinterpret_cast<uint32_t*>(q);
  q += (size_t)nseg_cap * 4;
  a.pre = reinterpret_cast<uint32_t*>(q);
  q += (size_t)nseg_cap * 8;
  a.jump = reinterpret_cast<uint32_t*>(q);  // [levels + 1][nseg * kCand] of the current window
}

// Buffers for a window of `bytes` and a batch of `cap` frames (grown, never shrunk).
int32_t reserve(State* g, uint64_t bytes, uint32_t cap) {
  hipError_t e = hipSuccess;
  if (bytes > g->half) {
    drop_prefetch(g);
    (void)hipDeviceSynchronize();  // work still reading the old window
    for (uint8_t*& b : g->d_buf) {
      if (b) (void)hipFree(b);
      b = nullptr;
    }
    g->half = 0;
    g->win_valid = false;
    for (uint8_t*& b : g->d_buf) {
      e = hipMalloc(reinterpret_cast<void**>(&b), 2 * bytes + kPad);
      if (e != hipSuccess) return hip_fail("hipMalloc (window)", e);
    }
    g->half = bytes;
  }
  if (bytes > g->h_cap && g->reg_mode < 0) {
    if (g->h_stage) (void)hipHostFree(g->h_stage);
    g->h_stage = nullptr;
    e = hipHostMalloc(reinterpret_cast<void**>(&g->h_stage), bytes, hipHostMallocDefault);
    if (e != hipSuccess) return hip_fail("hipHostMalloc (window)", e);
    g->h_cap = bytes;
  }
  const uint32_t nseg = (uint32_t)((2 * bytes + kSeg - 1) / kSeg);  // a window plus a moved tail
  if (nseg > g->seg_cap) {
    if (g->d_seg) (void)hipFree(g->d_seg);
    g->d_seg = nullptr;
    e = hipMalloc(reinterpret_cast<void**>(&g->d_seg), seg_bytes(nseg));
    if (e != hipSuccess) return hip_fail("hipMalloc (segments)", e);
    g->seg_cap = nseg;
  }
  if (cap > g->list_cap) {
    if (g->d_ptrs) (void)hipFree(g->d_ptrs);
    if (g->d_dl) (void)hipFree(g->d_dl);
    g->d_ptrs = nullptr;
    g->d_dl = nullptr;
    e = hipMalloc(reinterpret_cast<void**>(&g->d_ptrs), (size_t)cap * 8);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&g->d_dl), (size_t)cap * 2);
    if (e != hipSuccess) return hip_fail("hipMalloc (frame list)", e);
    g->list_cap = cap;
  }
  return RTN_OK;
}

// Starts copying the file bytes that follow the resident window into d_buf[1 - cur] + half, on
// cs after the work enqueued on s so far (it may still read that buffer). Registered mode only.
int32_t prefetch(rtn_pcap* p, State* g, hipStream_t s) {
  const uint64_t off = g->win_off + g->win_len;
  if (g->reg_mode <= 0 || off >= p->size) return RTN_OK;
  const uint64_t len = std::min<uint64_t>({g->window, p->size - off, g->half});
  uint8_t* dst = g->d_buf[1 - g->cur] + g->half;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p->base + off);
  const uintptr_t a1 = (a + 4095) & ~uintptr_t(4095), b1 = (a + len + 4095) & ~uintptr_t(4095);
  const uint64_t head = std::min<uint64_t>(len, a1 - a);  // inside the window's last registered page
  hipError_t e = hipEventRecord(g->s_ready, s);
  if (e == hipSuccess) e = hipStreamWaitEvent(g->cs, g->s_ready, 0);
  if (e == hipSuccess && len > head) {
    if (g->ahead.joinable()) g->ahead.join();
    if (g->ahead_lo == a1 && g->ahead_hi == b1 && g->ahead_ok) {
      g->ahead_ok = false;  // registered ahead: it becomes the prefetch's
    } else {
      drop_ahead(g);
      if (hipHostRegister(reinterpret_cast<void*>(a1), b1 - a1, hipHostRegisterReadOnly) != hipSuccess) {
        (void)hipGetLastError();
        return RTN_OK;  // no prefetch: the next window is copied when it is needed
      }
    }
    g->ahead_lo = g->ahead_hi = 0;
    g->pf_reg = reinterpret_cast<void*>(a1);
  }
  if (e == hipSuccess && head) e = hipMemcpyAsync(dst, p->base + off, head, hipMemcpyHostToDevice, g->cs);
  if (e == hipSuccess && len > head)
    e = hipMemcpyAsync(dst + head, p->base + off + head, len - head, hipMemcpyHostToDevice, g->cs);
  if (e == hipSuccess) e = hipMemsetAsync(dst + len, 0, kPad, g->cs);
  if (e == hipSuccess) e = hipEventRecord(g->pf_done, g->cs);
  if (e != hipSuccess) return hip_fail("window prefetch", e);
  g->pf_valid = true;
  g->pf_off = off;
  g->pf_len = len;
  // the window after this one starts at off + len: register its pages (past b1) meanwhile
  const uint64_t off2 = off + len;
  if (off2 < p->size) {
    const uint64_t len2 = std::min<uint64_t>({g->window, p->size - off2, g->half});
    const uintptr_t c = reinterpret_cast<uintptr_t>(p->base + off2);
    const uintptr_t lo = (c + 4095) & ~uintptr_t(4095), hi = (c + len2 + 4095) & ~uintptr_t(4095);
    drop_ahead(g);
    if (hi > lo && lo >= b1) {
      g->ahead_lo = lo;
      g->ahead_hi = hi;
      const int dev = g->device;
      g->ahead = std::thread([g, dev, lo, hi] {
        (void)hipSetDevice(dev);
        g->ahead_ok = hipHostRegister(reinterpret_cast<void*>(lo), hi - lo, hipHostRegisterReadOnly) == hipSuccess;
        if (!g->ahead_ok) (void)hipGetLastError();
      });
    }
  }
  return RTN_OK;
}

// file bytes [off, off + len) -> pinned staging, on worker threads (the first touch of each page
// of the mapping is read from the page cache here)
void copy_in(const uint8_t* src, uint8_t* dst, size_t len) {
  const unsigned hw = std::thread::hardware_concurrency();
  const size_t parts = std::min<size_t>(std::max(1u, std::min(hw, 12u)), std::max<size_t>(1, len >> 20));
  if (parts <= 1) {
    memcpy(dst, src, len);
    return;
  }
  const size_t step = ((len + parts - 1) / parts + 63) & ~size_t(63);
  std::vector<std::thread> th;
  for (size_t k = 0; k < parts; ++k) {
    const size_t a = k * step, b = std::min(len, a + step);
    if (a >= b) break;
    th.emplace_back([=] { memcpy(dst + a, src + a, b - a); });
  }
  for (auto& t : th) t.join();
}
}  // namespace rtn_gpu_walk

extern "C" {

int32_t rtn_pcap_gpu_window(rtn_pcap_t* p, uint64_t bytes) {
  if (!p) return rtn::set_error(RTN_EINVAL, "null argument");
  if (bytes < (1u << 16) || bytes > (1ull << 40)) return rtn::set_error(RTN_EINVAL, "window of 64 KiB .. 1 TiB");
  if (!p->gpu) p->gpu = new rtn_gpu_walk::State();
  p->gpu->window = bytes;
  p->gpu->win_valid = false;  // (an outstanding prefetch is dropped at the next batch)
  return RTN_OK;
}

int32_t rtn_pcap_next_batch_gpu(rtn_pcap_t* p, int device, const rtn_stage_slab_t* slab, uint32_t* n, void* stream) {
  using namespace rtn_gpu_walk;
  if (!p || !slab || !n) return rtn::set_error(RTN_EINVAL, "null argument");
  *n = 0;
  if (!slab->head || !slab->ext || !slab->ext_chunk || !slab->data_len || slab->cap == 0)
    return rtn::set_error(RTN_EINVAL, "null argument");
  if (slab->cap > RTN_MAX_FRAMES) return rtn::set_error(RTN_EINVAL, "cap larger than RTN_MAX_FRAMES");
  if (slab->ext_cap < rtn_stage_gather_ext_rows(slab->cap))
    return rtn::set_error(RTN_ERANGE, "the gather layout needs rtn_stage_gather_ext_rows(cap) ext rows");
  if (((reinterpret_cast<uintptr_t>(slab->head) | reinterpret_cast<uintptr_t>(slab->ext)) & 15u) != 0)
    return rtn::set_error(RTN_EINVAL, "head and ext must be 16-byte aligned");
  if (!p->gpu) p->gpu = new State();
  State* g = p->gpu;
  if (g->device != device) {
    if (g->device >= 0) return rtn::set_error(RTN_EINVAL, "a capture walks on one device");
    int32_t rc = init(g, device);
    if (rc) return rc;
  }
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return hip_fail("hipSetDevice", e);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  e = hipStreamWaitEvent(s, g->packed, 0);  // the previous batch's packing, on whatever stream
  if (e != hipSuccess) return hip_fail("hipStreamWaitEvent", e);
  // pcapng: the section's byte order, from the first section header when walking from the start
  if (p->fmt == Fmt::Pcapng && p->off == p->first && p->size >= 12) {
    uint32_t bom;
    memcpy(&bom, p->base + 8, 4);
    p->swap = bom != 0x1A2B3C4Du;
  }
  const bool swap = p->swap;
  for (;;) {
    if (p->off >= p->size) return RTN_OK;  // end of file: *n = 0
    // the window: the resident one if this batch starts inside it with at least half of it (or
    // the rest of the file) left, otherwise a fresh copy from here
    const uint64_t want = std::min<uint64_t>(g->window, p->size - p->off);
    int32_t rc = reserve(g, std::min<uint64_t>(g->window, p->size - p->first), slab->cap);
    if (rc) return rc;
    bool fresh = !(g->win_valid && p->off >= g->win_off && p->off < g->win_off + g->win_len);
    if (!fresh) {  // the rest of the resident window, if it holds about a batch (the last one's bytes)
      const uint64_t left = g->win_off + g->win_len - p->off;
      fresh = left < std::max<uint64_t>(g->last_batch, 1u << 20) && g->win_off + g->win_len < p->size;
    }
    const size_t off0 = p->off;
    if (fresh && g->pf_valid) {
      // the prefetched bytes follow the window: move its unread tail in front of them
      const bool follows = g->win_valid && g->pf_off == g->win_off + g->win_len && p->off >= g->win_off &&
                           p->off <= g->pf_off && g->pf_off - p->off <= g->half;
      if (follows) {
        const uint64_t tail = g->pf_off - p->off;
        uint8_t* nb = g->d_buf[1 - g->cur] + g->half - tail;
        e = hipEventSynchronize(g->pf_done);  // (the prefetch's first page is read through reg)
        if (e == hipSuccess) e = hipStreamWaitEvent(s, g->pf_done, 0);
        if (e == hipSuccess && tail)
          e = hipMemcpyAsync(nb, g->win_ptr + (p->off - g->win_off), tail, hipMemcpyDeviceToDevice, s);
        if (e != hipSuccess) return hip_fail("window switch", e);
        if (g->pf_reg) {
          if (g->reg) (void)hipHostUnregister(g->reg);
          g->reg = g->pf_reg;
          g->pf_reg = nullptr;
        }
        g->pf_valid = false;
        g->cur = 1 - g->cur;
        g->win_ptr = nb;
        g->win_off = p->off;
        g->win_len = tail + g->pf_len;
        fresh = false;
        int32_t prc = prefetch(p, g, s);
        if (prc) return prc;
      } else {
        drop_prefetch(g);
      }
    }
    if (fresh) {
      drop_ahead(g);  // (its pages may overlap this window's)
      prefault(p, p->off, want);
      e = hipEventSynchronize(g->copied);  // the previous window's copy has left its source
      if (e != hipSuccess) return hip_fail("hipEventSynchronize", e);
      if (g->reg) {  // the previous window's pages
        (void)hipHostUnregister(g->reg);
        g->reg = nullptr;
      }
      g->win_ptr = g->d_buf[g->cur] + g->half;
      e = hipSuccess;
      if (g->reg_mode > 0) {  // page-aligned cover of [off, off + want) inside the mapping
        const uintptr_t b0 = reinterpret_cast<uintptr_t>(p->base + p->off) & ~uintptr_t(4095);
        const uintptr_t b1 = (reinterpret_cast<uintptr_t>(p->base + p->off + want) + 4095) & ~uintptr_t(4095);
        e = hipHostRegister(reinterpret_cast<void*>(b0), b1 - b0, hipHostRegisterReadOnly);
        if (e == hipSuccess) {
          g->reg = reinterpret_cast<void*>(b0);
          e = hipMemcpyAsync(g->win_ptr, p->base + p->off, want, hipMemcpyHostToDevice, s);
        } else {
          (void)hipGetLastError();
          g->reg_mode = -1;
          e = hipSuccess;
          rc = reserve(g, std::min<uint64_t>(g->window, p->size - p->first), slab->cap);  // the staging buffer
          if (rc) return rc;
        }
      }
      // 16-MiB pieces: the host copies piece k + 1 while the copy engine moves piece k
      constexpr uint64_t kPiece = 16ull << 20;
      for (uint64_t a0 = 0; g->reg_mode < 0 && a0 < want && e == hipSuccess; a0 += kPiece) {
        const uint64_t len = std::min(kPiece, want - a0);
        copy_in(p->base + p->off + a0, g->h_stage + a0, len);
        e = hipMemcpyAsync(g->win_ptr + a0, g->h_stage + a0, len, hipMemcpyHostToDevice, s);
      }
      if (e == hipSuccess) e = hipEventRecord(g->copied, s);
      if (e == hipSuccess) e = hipMemsetAsync(g->win_ptr + want, 0, kPad, s);
      if (e != hipSuccess) return hip_fail("window copy", e);
      g->win_off = p->off;
      g->win_len = want;
      g->win_valid = true;
      rc = prefetch(p, g, s);
      if (rc) return rc;
    }
    const uint64_t rel = p->off - g->win_off, bytes = g->win_len - rel;
    const bool at_eof = g->win_off + g->win_len == p->size;
    // The walk covers the bytes the batch is expected to need (the last batch's file bytes per
    // packed frame, with a margin) when that is less than the window; its answer is taken only
    // if it holds more than `cap` kept frames (so it equals the whole window's), else the whole
    // window is walked.
    uint64_t lim = bytes;
    if (g->bpf > 0) {
      const double est = g->bpf * slab->cap * 1.25 + (256u << 10);
      if (est < (double)bytes) lim = std::min<uint64_t>(bytes, ((uint64_t)est + kSeg - 1) & ~(kSeg - 1));
    }
    CapArgs a{};
    Res r{};
    for (;;) {
      a = CapArgs{};
      a.win = g->win_ptr + rel;
      a.bytes = lim;
      a.nseg = (uint32_t)((lim + kSeg - 1) / kSeg);
      a.fmt = p->fmt == Fmt::Pcapng ? 1u : 0u;
      a.swap = swap ? 1u : 0u;
      a.mtu = p->mtu;
      a.at_eof = at_eof && lim == bytes ? 1u : 0u;
      carve(g->d_seg, g->seg_cap, a);
      a.levels = levels(a.nseg);
      a.red = g->d_res->red;
      a.tgt = g->d_res->tgt;
      a.cut = g->d_res->cut;
      a.cap = slab->cap;
      a.ptrs = g->d_ptrs;
      a.dlen = g->d_dl;
      void* params[] = {&a};
      e = hipMemsetAsync(g->d_res, 0, sizeof(Res), s);
      const uint32_t nb4 = (a.nseg + 3) / 4, nb256 = (a.nseg + 255) / 256, nbn = (a.nseg * kCand + 255) / 256;
      if (e == hipSuccess) e = hipModuleLaunchKernel(g->cand, nb4, 1, 1, 256, 1, 1, 0, s, params, nullptr);
      if (e == hipSuccess) e = hipModuleLaunchKernel(g->nodes, nbn, 1, 1, 256, 1, 1, 0, s, params, nullptr);
      for (uint32_t k = 1; k <= a.levels && e == hipSuccess; ++k) {
        a.k = k;  // (the launch copies the arguments)
        e = hipModuleLaunchKernel(g->jump, nbn, 1, 1, 256, 1, 1, 0, s, params, nullptr);
      }
      if (e == hipSuccess) e = hipModuleLaunchKernel(g->lift, nb256, 1, 1, 256, 1, 1, 0, s, params, nullptr);
      if (e == hipSuccess) e = hipModuleLaunchKernel(g->scan, 1, 1, 1, 1024, 1, 1, 0, s, params, nullptr);
      if (e == hipSuccess) e = hipModuleLaunchKernel(g->emit, nb256, 1, 1, 256, 1, 1, 0, s, params, nullptr);
      if (e == hipSuccess) e = hipMemcpyAsync(g->h_res, g->d_res, sizeof(Res), hipMemcpyDeviceToHost, s);
      if (e == hipSuccess) e = hipStreamSynchronize(s);
      if (e != hipSuccess) return hip_fail("rtn_pcap_next_batch_gpu", e);
      r = *g->h_res;
      if (lim == bytes || (r.tgt[0] == slab->cap && r.red[3] > slab->cap)) break;
      lim = bytes;
    }
    const uint32_t recs = r.red[2], kept = r.red[3], tgt = r.tgt[0], bad = r.tgt[1];
    const uint64_t ex = r.cut[2];
    // a pcapng section in the other byte order: the frames before it, then the error at it
    const bool order = (ex & kStop) && (ex & kErr) && tgt == kept;
    if (order && tgt == 0)
      return rtn::set_error(RTN_EINVAL, "pcapng sections in different byte orders: use rtn_pcap_next_batch_split");
    if (tgt < kept) {  // cut by cap or by a frame longer than 65535 bytes
      p->off += r.cut[0];
      p->st.frames += r.cut[1];
      p->st.skipped_mtu += r.cut[1] - tgt;
    } else {
      p->st.frames += recs;
      p->st.skipped_mtu += recs - kept;
      if ((ex & kDead) || order) {  // the chain reached a record no candidate matched (or the
        p->off += ex & kOffMask;      // section header): the next batch starts there
      } else if (!(ex & kStop)) {
        p->off += bytes;
      } else if ((ex & kEof) || at_eof) {
        p->off = p->size;  // the capture ends here, as the host reader ends
      } else if ((ex & kOffMask) == 0) {
        return rtn::set_error(RTN_ERANGE, "a record larger than the GPU window (rtn_pcap_gpu_window)");
      } else {
        p->off += ex & kOffMask;
      }
    }
    p->st.packed += tgt;
    p->st.bytes += r.cut[3];
    g->last_batch = p->off - off0;
    if (tgt > 0) g->bpf = (double)g->last_batch / tgt;
    if (tgt > 0) {
      PackArgs pa{g->d_ptrs, g->d_dl, slab->head, slab->ext, slab->ext_chunk, slab->data_len, tgt};
      void* pp[] = {&pa};
      const uint32_t chunks = (tgt + RTN_CHUNK_FRAMES - 1) / RTN_CHUNK_FRAMES;
      e = hipModuleLaunchKernel(g->pack, (chunks + 3) / 4, 1, 1, 256, 1, 1, 0, s, pp, nullptr);
      if (e == hipSuccess) e = hipEventRecord(g->packed, s);
      if (e != hipSuccess) return hip_fail("rtn_cap_pack", e);
      *n = tgt;
    }
    if (bad == tgt && bad < kept) return rtn::set_error(RTN_ERANGE, "captured frame longer than 65535 bytes");
    if (tgt > 0) return RTN_OK;
    // every frame of the window was skipped: go on with the next one
  }
}

}  // extern "C"
