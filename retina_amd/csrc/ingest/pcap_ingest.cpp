// Offline ingest: libpcap / pcapng capture -> slot slab + data_len, the host side of the batched
// packet stage (include/retina_ingest.h). Reference behaviour: core/src/runtime/offline.rs:64-82
// (read every frame, skip frames whose original length exceeds the mtu, mbuf data = captured
// bytes) and core/src/memory/mbuf.rs:56-76 (Mbuf::from_bytes). The file is memory-mapped and
// walked once; packing is a bounded memcpy per frame.
#include "retina_ingest.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <string>

#include "../runtime/rtn_error.hpp"
#include "retina_pc.h"

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
  if (p->base) munmap(const_cast<uint8_t*>(p->base), p->size);
  delete p;
}

}  // extern "C"
