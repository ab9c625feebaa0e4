// C++ host side of the packet stage: a mirror of Retina's `Subscription`
// (core/src/subscription/mod.rs) over the C ABI of retina_pc.h, for hosts written in C++ (the
// reference is Rust; this is the layer its RX loop would call through the binding of
// INTEGRATION.md). Header-only, C++17, HIP runtime API for device memory.
//
//   retina::Subscription sub(spec_toml, device);     Subscription::new(filter()) (mod.rs:81-92):
//                                                    the spec compiled by filtergen, loaded on a GPU
//   retina::Burst b = sub.run(batch, stream);        continue_packet for every frame of a burst
//                                                    (mod.rs:125-127) plus process_packet's
//                                                    PacketContinue gate and L4Context::new (:94-116)
//   b.continue_packet(i)                             Actions.data of frame i
//   b.process_packets(f)                             f(idx, L4Context) for the frames process_packet
//                                                    hands to conn_tracker.process, in frame order
//   b.packet_callbacks(f)                            f(idx, site) for each ZcFrame / Payload callback
//                                                    the generated packet_continue ran inline
//                                                    (filtergen/src/data.rs:299-331), in call order
//   sub.stats()                                      the counters of core/src/stats/mod.rs:9-27 that
//                                                    rx_core.rs:127-139 and process_packet update
//
// Errors throw: retina::FilterError for a spec filtergen would refuse (RTN_EFILTER), and
// retina::RetinaError for any other C ABI failure (its code is the RTN_E* value). There is no CPU
// path: results come from the gfx950 kernel.
#ifndef RETINA_SUBSCRIPTION_HPP
#define RETINA_SUBSCRIPTION_HPP

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "retina_pc.h"

namespace retina {

class RetinaError : public std::runtime_error {
 public:
  RetinaError(int32_t code, const std::string& what) : std::runtime_error(what), code(code) {}
  int32_t code;
};

class FilterError : public RetinaError {
 public:
  using RetinaError::RetinaError;
};

inline void check(int32_t rc) {
  if (rc == RTN_OK) return;
  const char* e = rtn_last_error();
  const std::string msg = e ? e : "retina error";
  if (rc == RTN_EFILTER) throw FilterError(rc, msg);
  throw RetinaError(rc, msg);
}

inline void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw RetinaError(RTN_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

constexpr uint32_t kPacketContinue = 1u;  // ActionData::PacketContinue (core/src/filter/actions.rs:17-76)

// std::net::SocketAddr: ip in network byte order (4 bytes used for IPv4), port in host order.
struct SocketAddr {
  bool v6 = false;
  uint8_t ip[16] = {};
  uint16_t port = 0;
};

// core/src/conntrack/pdu.rs:66-84
struct L4Context {
  SocketAddr src, dst;
  size_t proto = 0;
  size_t offset = 0;
  size_t length = 0;
  uint32_t seq_no = 0;
  uint32_t ack_no = 0;
  uint8_t flags = 0;
};

// core/src/stats/mod.rs:9-27 (the packet-stage ones)
struct Stats {
  uint64_t TOTAL_PKT = 0, TOTAL_BYTE = 0;
  uint64_t IGNORED_BY_PACKET_FILTER_PKT = 0, IGNORED_BY_PACKET_FILTER_BYTE = 0;
  uint64_t TCP_PKT = 0, TCP_BYTE = 0, UDP_PKT = 0, UDP_BYTE = 0;
  Stats& operator+=(const Stats& o) {
    TOTAL_PKT += o.TOTAL_PKT; TOTAL_BYTE += o.TOTAL_BYTE;
    IGNORED_BY_PACKET_FILTER_PKT += o.IGNORED_BY_PACKET_FILTER_PKT;
    IGNORED_BY_PACKET_FILTER_BYTE += o.IGNORED_BY_PACKET_FILTER_BYTE;
    TCP_PKT += o.TCP_PKT; TCP_BYTE += o.TCP_BYTE; UDP_PKT += o.UDP_PKT; UDP_BYTE += o.UDP_BYTE;
    return *this;
  }
};

// One packet-level callback site of the generated code (statement k of a deliver mask).
struct CallbackSite {
  uint32_t subscription;  // index in the spec
  std::string callback;   // the subscription's callback
  bool payload;           // Payload (true) or ZcFrame datatype
};

class Subscription;

// The results of one Subscription::run, on the host.
class Burst {
 public:
  size_t n() const { return n_; }
  uint32_t core_id() const { return core_id_; }

  // Actions.data continue_packet returned for frame i (PacketContinue or nothing at this layer,
  // core/src/filter/datatypes.rs:618-638).
  uint32_t continue_packet(size_t i) const { return bit(pc_, i) ? kPacketContinue : 0u; }

  // f(frame index, const L4Context&) for every forwarded frame, in frame order.
  template <class F>
  void process_packets(F&& f) const {
    const size_t nch = (n_ + RTN_CHUNK_FRAMES - 1) / RTN_CHUNK_FRAMES;
    for (size_t c = 0; c < nch; ++c) {
      uint32_t k = 0, k6 = 0, kt = 0;  // records, IPv6 records, TCP records of chunk c
      for (size_t i = c * RTN_CHUNK_FRAMES; i < n_ && i < (c + 1) * RTN_CHUNK_FRAMES; ++i) {
        if (!bit(fwd_, i)) continue;
        const rtn_l4ctx_t& r = l4_[RTN_REC_INDEX(n_, c, k)];
        L4Context x;
        x.proto = RTN_L4_PROTO(r.meta);
        x.offset = RTN_L4_OFFSET(r.meta);
        x.length = RTN_L4_LENGTH(r.meta);
        x.flags = (uint8_t)RTN_L4_FLAGS(r.meta);
        x.src.port = (uint16_t)(r.ports & 0xFFFFu);
        x.dst.port = (uint16_t)(r.ports >> 16);
        const bool tcp = x.proto == 6;
        if (RTN_L4_IPV6(r.meta)) {  // source bytes 0..7 in the record, the other 24 B in addr6
          const uint8_t* a = &addr6_[(c * RTN_CHUNK_FRAMES + k6) * 24u];
          x.src.v6 = x.dst.v6 = true;
          std::memcpy(x.src.ip, &r.w0, 4);
          std::memcpy(x.src.ip + 4, &r.w1, 4);
          std::memcpy(x.src.ip + 8, a, 8);
          std::memcpy(x.dst.ip, a + 8, 16);
          ++k6;
        } else {
          for (int j = 0; j < 4; ++j) {
            x.src.ip[j] = (uint8_t)(r.w0 >> (24 - 8 * j));
            x.dst.ip[j] = (uint8_t)(r.w1 >> (24 - 8 * j));
          }
        }
        if (tcp) {  // the seqack side stream, ranked among the chunk's TCP records
          const uint64_t t = seqack_[RTN_REC_INDEX(n_, c, kt)];
          x.seq_no = RTN_SEQACK_SEQ(t);
          x.ack_no = RTN_SEQACK_ACK(t);
          ++kt;
        }
        f(i, x);
        ++k;
      }
    }
  }

  // f(frame index, const CallbackSite&) for each packet-level callback the generated
  // packet_continue ran: frames in order, a frame's callbacks in code order.
  template <class F>
  void packet_callbacks(F&& f) const {
    if (words_ == 0) return;
    const size_t nch = (n_ + RTN_CHUNK_FRAMES - 1) / RTN_CHUNK_FRAMES;
    for (size_t c = 0; c < nch; ++c) {
      size_t k = 0;
      for (size_t i = c * RTN_CHUNK_FRAMES; i < n_ && i < (c + 1) * RTN_CHUNK_FRAMES; ++i) {
        if (!bit(dlv_, i)) continue;
        const uint64_t* m = &dlv_recs_[(c * RTN_CHUNK_FRAMES + k) * words_];
        for (size_t s = 0; s < sites_->size(); ++s)
          if ((m[s / 64] >> (s % 64)) & 1ull) f(i, (*sites_)[s]);
        ++k;
      }
    }
  }

  const Stats& stats() const { return stats_; }

 private:
  friend class Subscription;
  static bool bit(const std::vector<uint64_t>& bm, size_t i) { return (bm[i / 64] >> (i % 64)) & 1ull; }
  size_t n_ = 0;
  uint32_t core_id_ = 0;
  uint32_t words_ = 0;
  std::vector<uint64_t> pc_, fwd_, dlv_, dlv_recs_;
  std::vector<rtn_l4ctx_t> l4_;
  std::vector<uint64_t> seqack_;
  std::vector<uint8_t> addr6_;
  const std::vector<CallbackSite>* sites_ = nullptr;
  Stats stats_;
};

// One compiled subscription set loaded on one GPU; one per RX core, like the reference's
// per-lcore use. Not thread-safe (a context per thread).
class Subscription {
 public:
  Subscription(const std::string& spec_toml, int device = 0) : device_(device) {
    // a constructor that throws runs no destructor: release what was created before rethrowing
    try {
      check(rtn_program_compile(spec_toml.data(), spec_toml.size(), &prog_));
      check(rtn_program_info(prog_, &info_));
      const uint32_t ns = info_.n_deliver_stmts;
      std::vector<uint32_t> subs(ns ? ns : 1);
      std::vector<uint8_t> pay(ns ? ns : 1);
      check(rtn_program_deliver_table(prog_, subs.data(), pay.data(), ns ? ns : 1));
      for (uint32_t k = 0; k < ns; ++k) {
        std::string cb(rtn_program_deliver_callback(prog_, k, nullptr, 0), '\0');
        rtn_program_deliver_callback(prog_, k, &cb[0], cb.size() + 1);
        sites_.push_back({subs[k], cb, pay[k] != 0});
      }
      check(rtn_pc_create_from_program(prog_, device, &pc_));
    } catch (...) {
      if (pc_) rtn_pc_destroy(pc_);
      if (prog_) rtn_program_destroy(prog_);
      pc_ = nullptr;
      prog_ = nullptr;
      throw;
    }
  }
  Subscription(const Subscription&) = delete;
  Subscription& operator=(const Subscription&) = delete;
  ~Subscription() {
    release();
    if (pc_) rtn_pc_destroy(pc_);
    if (prog_) rtn_program_destroy(prog_);
  }

  const rtn_program_info_t& info() const { return info_; }
  const std::vector<CallbackSite>& callback_sites() const { return sites_; }
  const Stats& stats() const { return stats_; }

  // One burst through the packet stage: `in` points at device memory in the layout of
  // retina_pc.h. Synchronizes `stream`, accumulates stats() and throws if a frame's headers did
  // not fit its slot (RTN_STATUS_*: the results would not be the reference's).
  Burst run(const rtn_batch_t& in, hipStream_t stream = nullptr) {
    check_hip(hipSetDevice(device_), "hipSetDevice");
    reserve(in.n);
    rtn_pc_out_t o{};
    o.pc_bitmap = d_pc_;
    o.fwd_bitmap = d_fwd_;
    o.l4 = reinterpret_cast<rtn_l4ctx_t*>(d_l4_);
    o.addr6 = d_addr6_;
    o.seqack = d_seqack_;
    o.dlv_bitmap = info_.deliver_words ? d_dlv_ : nullptr;
    o.dlv_records = info_.deliver_words ? d_dlv_recs_ : nullptr;
    o.counters = d_counters_;
    check(rtn_pc_run(pc_, &in, &o, stream));
    Burst b;
    b.n_ = in.n;
    b.core_id_ = in.core_id;
    b.words_ = info_.deliver_words;
    b.sites_ = &sites_;
    const size_t bm = rtn_out_bitmap_bytes(in.n);
    b.pc_.resize(bm / 8);
    b.fwd_.resize(bm / 8);
    b.l4_.resize(rtn_out_l4_bytes(in.n) / sizeof(rtn_l4ctx_t));
    b.addr6_.resize(rtn_out_addr6_bytes(in.n));
    b.seqack_.resize(rtn_out_seqack_bytes(in.n) / 8);
    uint32_t cnt[RTN_COUNTERS_BYTES / 4];
    d2h(b.pc_.data(), d_pc_, bm, stream);
    d2h(b.fwd_.data(), d_fwd_, bm, stream);
    d2h(b.l4_.data(), d_l4_, b.l4_.size() * sizeof(rtn_l4ctx_t), stream);
    d2h(b.addr6_.data(), d_addr6_, b.addr6_.size(), stream);
    d2h(b.seqack_.data(), d_seqack_, b.seqack_.size() * 8, stream);
    d2h(cnt, d_counters_, sizeof(cnt), stream);
    if (info_.deliver_words) {
      b.dlv_.resize(bm / 8);
      b.dlv_recs_.resize(rtn_out_dlv_bytes(in.n, info_.deliver_words) / 8);
      d2h(b.dlv_.data(), d_dlv_, bm, stream);
      d2h(b.dlv_recs_.data(), d_dlv_recs_, b.dlv_recs_.size() * 8, stream);
    }
    check_hip(hipStreamSynchronize(stream), "hipStreamSynchronize");
    if (cnt[RTN_CNT_STATUS])
      throw RetinaError(RTN_EINVAL, "frames whose headers do not fit their slots (status " +
                                        std::to_string(cnt[RTN_CNT_STATUS]) + ")");
    auto u64 = [&](uint32_t w) { uint64_t v; std::memcpy(&v, &cnt[w], 8); return v; };
    Stats& s = b.stats_;
    s.TOTAL_PKT = in.n;
    s.TOTAL_BYTE = u64(RTN_CNT_TOTAL_BYTE);
    s.IGNORED_BY_PACKET_FILTER_PKT = in.n - cnt[RTN_CNT_PC];
    s.IGNORED_BY_PACKET_FILTER_BYTE = u64(RTN_CNT_IGNORED_BYTE);
    s.TCP_PKT = cnt[RTN_CNT_TCP_PKT];
    s.UDP_PKT = cnt[RTN_CNT_UDP_PKT];
    s.TCP_BYTE = u64(RTN_CNT_TCP_BYTE);
    s.UDP_BYTE = u64(RTN_CNT_UDP_BYTE);
    stats_ += s;
    return b;
  }

 private:
  static void d2h(void* dst, const void* src, size_t bytes, hipStream_t s) {
    if (bytes) check_hip(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
  }
  static void* dalloc(size_t bytes) {
    void* p = nullptr;
    check_hip(hipMalloc(&p, bytes ? bytes : 64), "hipMalloc");
    return p;
  }
  void release() {
    for (void* p : {static_cast<void*>(d_pc_), static_cast<void*>(d_fwd_), d_l4_, static_cast<void*>(d_addr6_),
                    static_cast<void*>(d_seqack_), static_cast<void*>(d_dlv_), static_cast<void*>(d_dlv_recs_),
                    static_cast<void*>(d_counters_)})
      if (p) (void)hipFree(p);
    d_pc_ = d_fwd_ = d_dlv_ = d_dlv_recs_ = d_seqack_ = nullptr;
    d_l4_ = nullptr;
    d_addr6_ = nullptr;
    d_counters_ = nullptr;
    cap_ = 0;
  }
  void reserve(uint32_t n) {
    if (n <= cap_ && d_counters_) return;
    release();
    d_pc_ = static_cast<uint64_t*>(dalloc(rtn_out_bitmap_bytes(n)));
    d_fwd_ = static_cast<uint64_t*>(dalloc(rtn_out_bitmap_bytes(n)));
    d_l4_ = dalloc(rtn_out_l4_bytes(n));
    d_addr6_ = static_cast<uint8_t*>(dalloc(rtn_out_addr6_bytes(n)));
    d_seqack_ = static_cast<uint64_t*>(dalloc(rtn_out_seqack_bytes(n)));
    if (info_.deliver_words) {
      d_dlv_ = static_cast<uint64_t*>(dalloc(rtn_out_bitmap_bytes(n)));
      d_dlv_recs_ = static_cast<uint64_t*>(dalloc(rtn_out_dlv_bytes(n, info_.deliver_words)));
    }
    d_counters_ = static_cast<uint32_t*>(dalloc(RTN_COUNTERS_BYTES));
    cap_ = n;
  }

  int device_;
  rtn_program_t* prog_ = nullptr;
  rtn_pc_t* pc_ = nullptr;
  rtn_program_info_t info_{};
  std::vector<CallbackSite> sites_;
  Stats stats_;
  uint32_t cap_ = 0;
  uint64_t *d_pc_ = nullptr, *d_fwd_ = nullptr, *d_dlv_ = nullptr, *d_dlv_recs_ = nullptr, *d_seqack_ = nullptr;
  void* d_l4_ = nullptr;
  uint8_t* d_addr6_ = nullptr;
  uint32_t* d_counters_ = nullptr;
};

}  // namespace retina

#endif  // RETINA_SUBSCRIPTION_HPP
