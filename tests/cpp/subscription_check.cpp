// Drives include/retina_subscription.hpp (the C++ Subscription mirror) on one GPU for
// tests/test_subscription.py: reads a spec, a slab of 128-B slots and their data_len, runs one
// burst, and prints what the reference's Subscription would have done, one fact per line:
//   pc <i>                          continue_packet(i) has PacketContinue
//   l4 <i> <src> <sport> <dst> <dport> <proto> <offset> <length> <seq> <ack> <flags>
//   cb <i> <subscription> <callback> <ZcFrame|Payload>
//   stat <NAME> <value>
// Usage: subscription_check <spec.toml> <slab.bin> <dlen.bin> [device]
#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "retina_subscription.hpp"

static std::string slurp(const char* path) {
  std::ifstream in(path, std::ios::binary);
  std::stringstream ss;
  ss << in.rdbuf();
  return ss.str();
}

static void ip(const retina::SocketAddr& a) {
  if (a.v6) {
    for (int j = 0; j < 16; ++j) std::printf("%02x", a.ip[j]);
  } else {
    std::printf("%u.%u.%u.%u", a.ip[0], a.ip[1], a.ip[2], a.ip[3]);
  }
}

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s spec.toml slab.bin dlen.bin [device]\n", argv[0]);
    return 2;
  }
  const int device = argc > 4 ? std::atoi(argv[4]) : 0;
  try {
    const std::string spec = slurp(argv[1]), slab = slurp(argv[2]), dl = slurp(argv[3]);
    const uint32_t n = (uint32_t)(dl.size() / 2);
    if (slab.size() != (size_t)n * 128u) throw retina::RetinaError(RTN_EINVAL, "slab is not n 128-B slots");
    retina::Subscription sub(spec, device);
    void *d_slab = nullptr, *d_dlen = nullptr;
    retina::check_hip(hipMalloc(&d_slab, slab.size() ? slab.size() : 128), "hipMalloc");
    retina::check_hip(hipMalloc(&d_dlen, dl.size() ? dl.size() : 2), "hipMalloc");
    retina::check_hip(hipMemcpy(d_slab, slab.data(), slab.size(), hipMemcpyHostToDevice), "hipMemcpy");
    retina::check_hip(hipMemcpy(d_dlen, dl.data(), dl.size(), hipMemcpyHostToDevice), "hipMemcpy");
    rtn_batch_t b{};
    b.slab = static_cast<const uint8_t*>(d_slab);
    b.stride = 128;
    b.data_len = static_cast<const uint16_t*>(d_dlen);
    b.n = n;
    b.core_id = 3;
    retina::Burst r = sub.run(b);
    for (size_t i = 0; i < r.n(); ++i)
      if (r.continue_packet(i) & retina::kPacketContinue) std::printf("pc %zu\n", i);
    r.process_packets([](size_t i, const retina::L4Context& c) {
      std::printf("l4 %zu ", i);
      ip(c.src);
      std::printf(" %u ", c.src.port);
      ip(c.dst);
      std::printf(" %u %zu %zu %zu %u %u %u\n", c.dst.port, c.proto, c.offset, c.length, c.seq_no, c.ack_no, c.flags);
    });
    r.packet_callbacks([](size_t i, const retina::CallbackSite& s) {
      std::printf("cb %zu %u %s %s\n", i, s.subscription, s.callback.c_str(), s.payload ? "Payload" : "ZcFrame");
    });
    const retina::Stats& s = sub.stats();
    std::printf("stat TOTAL_PKT %llu\nstat TOTAL_BYTE %llu\nstat IGNORED_BY_PACKET_FILTER_PKT %llu\n"
                "stat IGNORED_BY_PACKET_FILTER_BYTE %llu\nstat TCP_PKT %llu\nstat TCP_BYTE %llu\n"
                "stat UDP_PKT %llu\nstat UDP_BYTE %llu\n",
                (unsigned long long)s.TOTAL_PKT, (unsigned long long)s.TOTAL_BYTE,
                (unsigned long long)s.IGNORED_BY_PACKET_FILTER_PKT, (unsigned long long)s.IGNORED_BY_PACKET_FILTER_BYTE,
                (unsigned long long)s.TCP_PKT, (unsigned long long)s.TCP_BYTE, (unsigned long long)s.UDP_PKT,
                (unsigned long long)s.UDP_BYTE);
    (void)hipFree(d_slab);
    (void)hipFree(d_dlen);
  } catch (const retina::FilterError& e) {
    std::fprintf(stderr, "FilterError %d: %s\n", e.code, e.what());
    return 3;
  } catch (const retina::RetinaError& e) {
    std::fprintf(stderr, "RetinaError %d: %s\n", e.code, e.what());
    return 4;
  }
  return 0;
}
