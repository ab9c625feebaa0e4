// PacketContinue code generation: the filtergen step of the reference, retargeted to HIP.
//
//   filtergen/src/packet_filter.rs:7-73   gen_packet_filter / gen_packet_filter_util
//   filtergen/src/utils.rs:18-249         binary_to_tokens (predicate -> expression)
//   filtergen/src/utils.rs:251-285        update_body (actions, then delivers)
//   filtergen/src/utils.rs:298-379        PacketDataFilter::{add_unary_pred, add_binary_pred, add_root_pred}
//   filtergen/src/data.rs:262-331         build_packet_callback (ZcFrame / Payload from_mbuf guards)
#pragma once

#include <string>
#include <vector>

#include "filter.hpp"

namespace rtn {

// One packet-level callback invocation site in the generated code, in code (= execution) order.
struct DeliverStmt {
  uint32_t sub_id;       // subscription index in the spec
  bool payload;          // Payload datatype: fires only if the payload slice is readable
  std::string callback;  // callback name (for the host dispatcher)
};

struct PacketProgram {
  std::vector<SubscriptionSpec> subs;
  PTree tree{FilterLayer::PacketContinue};
  std::vector<DeliverStmt> delivers;
  std::string hip_body;     // __device__ function rtn_filter(...) specialised to this tree
  std::string rust_listing; // the Rust the reference filtergen would emit (normalised), for review
  bool wraps_ethernet = false;
  uint32_t deliver_words() const { return (uint32_t)((delivers.size() + 63) / 64); }
};

// Compile subscriptions into the PacketContinue program. Throws FilterError on any filter
// the reference would reject at compile time (parse errors, layer errors, type errors).
PacketProgram compile_packet_program(const std::vector<SubscriptionSpec>& subs);

}  // namespace rtn
