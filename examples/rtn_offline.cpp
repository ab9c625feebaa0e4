// rtn_offline: the batched offline runtime (core/src/runtime/offline.rs:39-95) on the C ABI, in C++.
//
//   rtn_offline <spec.toml> <capture.pcap|pcapng> [--batch N] [--mtu M] [--device D] [--no-ct]
//               [--ct-log2 L] [--max-conn C] [--dump FILE] [--layout compact|mono]
//
// The reference's offline loop reads a capture frame by frame, skips frames longer than the
// mtu, wraps each in an Mbuf and calls Subscription::process_packet, which runs packet_continue,
// L4Context::new and ConnTracker::process. Here the same work runs per batch:
//
//   rtn_pcap_next_batch_split   capture -> pinned compact split layout: 64-B head slots + ext rows
//                         only for frames whose headers may pass byte 64 (offline.rs:64-75 rules;
//                         --layout mono: rtn_pcap_next_batch into 128-B slots)
//   hipMemcpyAsync        slab + data_len -> HBM
//   rtn_pc_run            packet_continue + L4Context::new + connection stage (one launch)
//   rtn_ct_process        the ConnTracker table step (two launches; HBM-resident table)
//   hipMemcpyAsync        bitmaps, L4Context records, connection entries -> host
//   host walk             forwarded frames in frame order, as ConnTracker::process sees them
//
// Two host buffer sets alternate, so the host reads batch i+1 and walks batch i-1 while the GPU
// works on batch i. GPU work stays on one stream: the table's batches must run in order.
// --dump writes one line per forwarded frame (frame index, 5-tuple, connection status) for the
// tests; stdout gets one JSON summary line (the offline runtime's counters plus throughput).
#include <hip/hip_runtime.h>

#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "retina_ct.h"
#include "retina_stage.h"
#include "retina_ingest.h"
#include "retina_pc.h"

namespace {

[[noreturn]] void die(const char* what, int32_t rc) {
  fprintf(stderr, "rtn_offline: %s failed (%d): %s\n", what, rc, rtn_last_error());
  exit(1);
}
#define RTN_CHECK(call)                  \
  do {                                   \
    int32_t rc_ = (call);                \
    if (rc_ != RTN_OK) die(#call, rc_);  \
  } while (0)
#define HIP_CHECK(call)                                                           \
  do {                                                                            \
    hipError_t e_ = (call);                                                       \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "rtn_offline: %s: %s\n", #call, hipGetErrorString(e_));    \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

template <typename T>
T* dev_alloc(size_t bytes) {
  void* p = nullptr;
  HIP_CHECK(hipMalloc(&p, bytes ? bytes : 16));
  return static_cast<T*>(p);
}
template <typename T>
T* host_alloc(size_t bytes) {
  void* p = nullptr;
  HIP_CHECK(hipHostMalloc(&p, bytes ? bytes : 16, hipHostMallocDefault));
  return static_cast<T*>(p);
}

constexpr uint64_t kStride = 128;  // every header the parse can reach (98 B max) fits

struct HostSet {  // one batch in flight: pinned input and result buffers
  uint8_t* slab;        // 128-B slots (mono) or 64-B head slots (compact)
  uint8_t* ext;         // compact: ext rows
  uint32_t* ext_chunk;  // compact: first row of each RTN_CHUNK_FRAMES-frame chunk
  uint32_t rows = 0;
  uint16_t* dlen;
  uint64_t* fwd;
  uint64_t* pcbm;
  rtn_l4ctx_t* l4;
  uint8_t* addr6;
  rtn_ct_entry_t* ct;
  uint32_t n = 0;
  uint64_t first_frame = 0;  // index of the batch's first frame in the capture
  bool pending = false;
};

struct Totals {
  uint64_t frames = 0, pc = 0, fwd = 0, tcp = 0, udp = 0;
  uint64_t status[8] = {};
  uint64_t prior = 0;
};

void walk(const HostSet& h, bool with_ct, Totals& t, FILE* dump) {
  const uint32_t words = (h.n + 63u) / 64u;
  for (uint32_t w = 0; w < words; ++w) t.pc += __builtin_popcountll(h.pcbm[w]);
  for (uint32_t c = 0; c * RTN_CHUNK_FRAMES < h.n; ++c) {
    uint32_t rank = 0;                                // forwarded frames of the chunk before this one
    uint64_t k6 = (uint64_t)c * RTN_CHUNK_FRAMES;     // IPv6 address index (dense per chunk)
    for (uint32_t w = c * (RTN_CHUNK_FRAMES / 64u); w < (c + 1) * (RTN_CHUNK_FRAMES / 64u) && w < words; ++w) {
      for (uint64_t b = h.fwd[w]; b; b &= b - 1, ++rank) {
        const uint64_t i = (uint64_t)w * 64u + __builtin_ctzll(b);
        const uint64_t k = RTN_REC_INDEX(h.n, c, rank);  // record index
        const rtn_l4ctx_t& r = h.l4[k];
        const bool v6 = RTN_L4_IPV6(r.meta);
        ++t.fwd;
        (RTN_L4_PROTO(r.meta) == 6 ? t.tcp : t.udp) += 1;
        uint32_t slot = RTN_CT_NO_SLOT, status = 0;
        if (with_ct) {
          slot = h.ct[k].slot;
          status = h.ct[k].status;
          t.status[status & 7u] += 1;
          t.prior += (status & RTN_CT_PRIOR) ? 1 : 0;
        }
        if (dump) {
          char src[40], dst[40];
          if (v6) {  // source bytes 0..7 in the record (w0, w1), the other 24 B in addr6
            const uint8_t* a = h.addr6 + k6 * 24u;
            uint8_t s0[8];
            std::memcpy(s0, &r.w0, 4);
            std::memcpy(s0 + 4, &r.w1, 4);
            char* p = src;
            for (int j = 0; j < 8; ++j) p += sprintf(p, "%02x", s0[j]);
            for (int j = 0; j < 8; ++j) p += sprintf(p, "%02x", a[j]);
            p = dst;
            for (int j = 8; j < 24; ++j) p += sprintf(p, "%02x", a[j]);
          } else {
            sprintf(src, "%08x", r.w0);  // an IPv4 record's addresses
            sprintf(dst, "%08x", r.w1);
          }
          fprintf(dump, "%llu %u %s %u %s %u %u %u\n", (unsigned long long)(h.first_frame + i), RTN_L4_PROTO(r.meta),
                  src, r.ports & 0xffffu, dst, r.ports >> 16, status, slot);
        }
        if (v6) ++k6;
      }
    }
  }
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: rtn_offline <spec.toml> <capture> [--batch N] [--mtu M] [--device D] [--no-ct] "
                    "[--ct-log2 L] [--max-conn C] [--dump FILE] [--layout compact|mono|gpu] [--window BYTES] [--one-stream] [--inline-results]\n");
    return 2;
  }
  uint32_t batch = 1u << 20, mtu = 9702, ct_log2 = 24, max_conn = 10000000;  // configs/offline.toml
  int device = 0;
  bool with_ct = true;
  const char* dump_path = nullptr;
  bool compact = true, gpu_walk = false, one_stream = false, inline_results = false;  // gpu: the capture walk on the GPU (rtn_pcap_next_batch_gpu)
  uint64_t window = 0;
  for (int a = 3; a < argc; ++a) {
    std::string s = argv[a];
    auto next = [&]() { return a + 1 < argc ? argv[++a] : (die("missing argument value", -22), nullptr); };
    if (s == "--batch") batch = (uint32_t)strtoul(next(), nullptr, 10);
    else if (s == "--mtu") mtu = (uint32_t)strtoul(next(), nullptr, 10);
    else if (s == "--device") device = atoi(next());
    else if (s == "--no-ct") with_ct = false;
    else if (s == "--ct-log2") ct_log2 = (uint32_t)strtoul(next(), nullptr, 10);
    else if (s == "--max-conn") max_conn = (uint32_t)strtoul(next(), nullptr, 10);
    else if (s == "--dump") dump_path = next();
    else if (s == "--layout") {
      const std::string l = next();
      if (l != "compact" && l != "mono" && l != "gpu") die("--layout compact|mono|gpu", -22);
      compact = l != "mono";
      gpu_walk = l == "gpu";
    }
    else if (s == "--window") window = strtoull(next(), nullptr, 10);
    else if (s == "--one-stream") one_stream = true;  // gpu: the walk on the stages' stream
    else if (s == "--inline-results") inline_results = true;  // results walked on the main thread
    else die(("unknown option " + s).c_str(), -22);
  }
  batch = (batch + RTN_CHUNK_FRAMES - 1) / RTN_CHUNK_FRAMES * RTN_CHUNK_FRAMES;

  std::ifstream f(argv[1]);
  if (!f) die("open spec", -2);
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string spec = ss.str();
  rtn_program_t* prog = nullptr;
  RTN_CHECK(rtn_program_compile(spec.data(), spec.size(), &prog));
  rtn_program_info_t info;
  RTN_CHECK(rtn_program_info(prog, &info));
  HIP_CHECK(hipSetDevice(device));
  rtn_pc_t* pc = nullptr;
  RTN_CHECK(rtn_pc_create_from_program(prog, device, &pc));
  rtn_ct_t* ct = nullptr;
  if (with_ct) RTN_CHECK(rtn_ct_create(device, ct_log2, max_conn, &ct));
  rtn_pcap_t* cap = nullptr;
  RTN_CHECK(rtn_pcap_open(argv[2], mtu, &cap));
  if (window) RTN_CHECK(rtn_pcap_gpu_window(cap, window));
  FILE* dump = dump_path ? fopen(dump_path, "w") : nullptr;

  // device buffers (one set: the stream orders the batches)
  const size_t bm = rtn_out_bitmap_bytes(batch), l4b = rtn_out_l4_bytes(batch), a6b = rtn_out_addr6_bytes(batch);
  const uint64_t stride = compact ? 64u : kStride;
  const uint32_t nchunks = batch / RTN_CHUNK_FRAMES;
  uint8_t* d_slab = dev_alloc<uint8_t>(batch * stride);
  uint8_t* d_ext = compact ? dev_alloc<uint8_t>((size_t)batch * 64u) : nullptr;
  uint32_t* d_chunk = compact ? dev_alloc<uint32_t>(nchunks * 4u) : nullptr;
  uint16_t* d_dlen = dev_alloc<uint16_t>(batch * 2u);
  rtn_pc_out_t out = {};
  out.pc_bitmap = dev_alloc<uint64_t>(bm);
  out.fwd_bitmap = dev_alloc<uint64_t>(bm);
  out.l4 = dev_alloc<rtn_l4ctx_t>(l4b);
  out.addr6 = dev_alloc<uint8_t>(a6b);
  if (info.deliver_words) {
    out.dlv_bitmap = dev_alloc<uint64_t>(bm);
    out.dlv_records = dev_alloc<uint64_t>(rtn_out_dlv_bytes(batch, info.deliver_words));
  }
  rtn_ct_entry_t* d_ct = nullptr;
  if (with_ct) {
    out.conn = dev_alloc<rtn_conn_t>(rtn_out_conn_bytes(batch));
    if (info.conn_words) out.conn_dlv = dev_alloc<uint64_t>(rtn_out_conn_dlv_bytes(batch, info.conn_words));
    d_ct = dev_alloc<rtn_ct_entry_t>(rtn_out_ct_bytes(batch));
  }
  // --layout gpu: the batch is packed on the device, so the device slab is the double buffer (the
  // walk of batch k + 1 runs on its own stream while batch k runs through the stages)
  uint8_t* g_slab[2] = {d_slab, nullptr};
  uint8_t* g_ext[2] = {d_ext, nullptr};
  uint32_t* g_chunk[2] = {d_chunk, nullptr};
  uint16_t* g_dlen[2] = {d_dlen, nullptr};
  hipStream_t wstream = nullptr;
  hipEvent_t walked = nullptr;
  if (gpu_walk) {
    g_slab[1] = dev_alloc<uint8_t>(batch * stride);
    g_ext[1] = dev_alloc<uint8_t>((size_t)batch * 64u);
    g_chunk[1] = dev_alloc<uint32_t>(nchunks * 4u);
    g_dlen[1] = dev_alloc<uint16_t>(batch * 2u);
    HIP_CHECK(hipStreamCreateWithFlags(&wstream, hipStreamNonBlocking));
    HIP_CHECK(hipEventCreateWithFlags(&walked, hipEventDisableTiming));
  }
  HostSet hs[2];
  for (auto& h : hs) {
    h.slab = host_alloc<uint8_t>(batch * stride);
    h.ext = compact ? host_alloc<uint8_t>((size_t)batch * 64u) : nullptr;
    h.ext_chunk = compact ? host_alloc<uint32_t>(nchunks * 4u) : nullptr;
    h.dlen = host_alloc<uint16_t>(batch * 2u);
    h.fwd = host_alloc<uint64_t>(bm);
    h.pcbm = host_alloc<uint64_t>(bm);
    h.l4 = host_alloc<rtn_l4ctx_t>(l4b);
    h.addr6 = host_alloc<uint8_t>(a6b);
    h.ct = with_ct ? host_alloc<rtn_ct_entry_t>(rtn_out_ct_bytes(batch)) : nullptr;
  }
  hipStream_t stream;
  HIP_CHECK(hipStreamCreate(&stream));
  hipEvent_t done[2];
  for (auto& e : done) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));

  Totals t;
  uint64_t next_frame = 0;
  double t_wait = 0, t_walk = 0, t_pack = 0;  // host time split (seconds)
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto secs_since = [&](std::chrono::steady_clock::time_point a) { return std::chrono::duration<double>(now() - a).count(); };
  // A results thread walks the batches in capture order (waiting for each one's event), so the
  // main thread only packs and enqueues; it waits for the thread before reusing a buffer set.
  std::mutex mu;
  std::condition_variable cv;
  std::deque<uint32_t> queue;
  bool stop = false;
  double r_wait = 0, r_walk = 0;  // the results thread's time
  std::thread results;
  if (!inline_results)
    results = std::thread([&] {
      for (;;) {
        uint32_t k;
        {
          std::unique_lock<std::mutex> l(mu);
          cv.wait(l, [&] { return stop || !queue.empty(); });
          if (queue.empty()) return;
          k = queue.front();
          queue.pop_front();
        }
        auto a = now();
        HIP_CHECK(hipEventSynchronize(done[k]));
        r_wait += secs_since(a);
        a = now();
        walk(hs[k], with_ct, t, dump);
        r_walk += secs_since(a);
        {
          std::lock_guard<std::mutex> l(mu);
          hs[k].pending = false;
        }
        cv.notify_all();
      }
    });
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t it = 0;; ++it) {
    HostSet& h = hs[it & 1u];
    if (!inline_results) {  // the results thread is done with batch it-2's buffers
      auto a = now();
      std::unique_lock<std::mutex> l(mu);
      cv.wait(l, [&] { return !h.pending; });
      t_wait += secs_since(a);
    } else if (h.pending) {  // results of batch it-2 (same buffers): wait, then walk them
      auto a = now();
      HIP_CHECK(hipEventSynchronize(done[it & 1u]));
      t_wait += secs_since(a);
      a = now();
      walk(h, with_ct, t, dump);
      t_walk += secs_since(a);
      h.pending = false;
    }
    uint32_t n = 0;
    const auto tp = now();
    if (gpu_walk) {  // the file's bytes to HBM, records found and frames packed by the GPU
      // (into the device set batch it - 2 used: its results were waited for above)
      d_slab = g_slab[it & 1u];
      d_ext = g_ext[it & 1u];
      d_chunk = g_chunk[it & 1u];
      d_dlen = g_dlen[it & 1u];
      rtn_stage_slab_t sl = {d_slab, d_ext, d_chunk, d_dlen, batch, batch};
      RTN_CHECK(rtn_pcap_next_batch_gpu(cap, device, &sl, &n, one_stream ? stream : wstream));
      if (!one_stream) {
        HIP_CHECK(hipEventRecord(walked, wstream));
        HIP_CHECK(hipStreamWaitEvent(stream, walked, 0));
      }
    } else if (compact) {
      RTN_CHECK(rtn_pcap_next_batch_split(cap, h.slab, h.ext, batch, h.ext_chunk, h.dlen, batch, &n, &h.rows));
    } else {
      RTN_CHECK(rtn_pcap_next_batch(cap, h.slab, kStride, h.dlen, batch, &n));
    }
    t_pack += secs_since(tp);
    if (n == 0) break;
    h.n = n;
    h.first_frame = next_frame;
    next_frame += n;
    t.frames += n;
    const size_t nbm = rtn_out_bitmap_bytes(n);
    rtn_batch_t b = {d_slab, stride, d_dlen, n, 0u, nullptr, 0u, 0u, nullptr};
    if (gpu_walk) {
      b.ext = d_ext;
      b.ext_rows = rtn_stage_gather_ext_rows(n);
      b.ext_chunk = d_chunk;
      b.flags = RTN_BATCH_EXT_COMPACT;
    } else {
      HIP_CHECK(hipMemcpyAsync(d_slab, h.slab, (size_t)n * stride, hipMemcpyHostToDevice, stream));
      HIP_CHECK(hipMemcpyAsync(d_dlen, h.dlen, (size_t)n * 2u, hipMemcpyHostToDevice, stream));
    }
    if (compact && !gpu_walk) {
      if (h.rows) HIP_CHECK(hipMemcpyAsync(d_ext, h.ext, (size_t)h.rows * 64u, hipMemcpyHostToDevice, stream));
      HIP_CHECK(hipMemcpyAsync(d_chunk, h.ext_chunk, ((n + RTN_CHUNK_FRAMES - 1) / RTN_CHUNK_FRAMES) * 4u,
                               hipMemcpyHostToDevice, stream));
      b.ext = d_ext;
      b.ext_rows = h.rows;
      b.ext_chunk = d_chunk;
      b.flags = RTN_BATCH_EXT_COMPACT;
    }
    RTN_CHECK(rtn_pc_run(pc, &b, &out, stream));
    if (with_ct) RTN_CHECK(rtn_ct_process(ct, &out, n, d_ct, stream));
    HIP_CHECK(hipMemcpyAsync(h.fwd, out.fwd_bitmap, nbm, hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipMemcpyAsync(h.pcbm, out.pc_bitmap, nbm, hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipMemcpyAsync(h.l4, out.l4, rtn_out_l4_bytes(n), hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipMemcpyAsync(h.addr6, out.addr6, rtn_out_addr6_bytes(n), hipMemcpyDeviceToHost, stream));
    if (with_ct) HIP_CHECK(hipMemcpyAsync(h.ct, d_ct, rtn_out_ct_bytes(n), hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipEventRecord(done[it & 1u], stream));
    if (!inline_results) {
      {
        std::lock_guard<std::mutex> l(mu);
        h.pending = true;
        queue.push_back(it & 1u);
      }
      cv.notify_all();
    } else {
      h.pending = true;
    }
  }
  if (!inline_results) {
    {
      std::lock_guard<std::mutex> l(mu);
      stop = true;
    }
    cv.notify_all();
    results.join();
    t_walk = r_walk;
  }
  for (uint32_t k = 0; k < 2; ++k) {
    if (!hs[k].pending) continue;
    HIP_CHECK(hipEventSynchronize(done[k]));
  }
  // walk the (at most two) outstanding batches in capture order
  int first = hs[0].pending && hs[1].pending ? (hs[0].first_frame < hs[1].first_frame ? 0 : 1) : (hs[0].pending ? 0 : 1);
  for (int k = 0; k < 2; ++k) {
    HostSet& h = hs[(first + k) & 1];
    if (h.pending) walk(h, with_ct, t, dump);
  }
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  rtn_pcap_stats_t ps;
  RTN_CHECK(rtn_pcap_stats(cap, &ps));
  rtn_ct_stats_t cs = {};
  if (with_ct) RTN_CHECK(rtn_ct_stats(ct, &cs));
  printf("{\"frames_read\": %llu, \"skipped_mtu\": %llu, \"frames\": %llu, \"bytes\": %llu, \"packet_continue\": %llu, "
         "\"forwarded\": %llu, \"tcp\": %llu, \"udp\": %llu, \"ct\": {\"hit\": %llu, \"new\": %llu, \"miss\": %llu, "
         "\"new_dropped\": %llu, \"full\": %llu, \"collision\": %llu, \"prior\": %llu, \"live\": %u}, "
         "\"seconds\": %.6f, \"mpps\": %.2f, \"batch\": %u, \"layout\": \"%s\", "
         "\"host_s\": {\"pack\": %.4f, \"wait\": %.4f, \"walk\": %.4f}}\n",
         (unsigned long long)ps.frames, (unsigned long long)ps.skipped_mtu, (unsigned long long)t.frames,
         (unsigned long long)ps.bytes, (unsigned long long)t.pc, (unsigned long long)t.fwd, (unsigned long long)t.tcp,
         (unsigned long long)t.udp, (unsigned long long)t.status[1], (unsigned long long)t.status[2],
         (unsigned long long)t.status[3], (unsigned long long)t.status[4], (unsigned long long)t.status[5],
         (unsigned long long)t.status[6], (unsigned long long)t.prior, cs.live, secs, t.frames / secs / 1e6, batch,
         gpu_walk ? "gpu" : (compact ? "compact" : "mono"), t_pack, t_wait,
         t_walk);
  if (dump) fclose(dump);
  rtn_pcap_close(cap);
  if (ct) rtn_ct_destroy(ct);
  rtn_pc_destroy(pc);
  rtn_program_destroy(prog);
  return 0;
}
