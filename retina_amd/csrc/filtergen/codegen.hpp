// PacketContinue code generation: the filtergen step of the reference, retargeted to HIP.
//
//   filtergen/src/packet_filter.rs:7-73   gen_packet_filter / gen_packet_filter_util
//   filtergen/src/utils.rs:18-249         binary_to_tokens (predicate -> expression)
//   filtergen/src/utils.rs:251-285        update_body (actions, then delivers)
//   filtergen/src/utils.rs:298-379        PacketDataFilter::{add_unary_pred, add_binary_pred, add_root_pred}
//   filtergen/src/data.rs:262-331         build_packet_callback (ZcFrame / Payload from_mbuf guards)
//   filtergen/src/deliver_filter.rs:9-151 gen_deliver_filter (FilterLayer::PacketDeliver)
#pragma once

#include <string>
#include <vector>

#include "filter.hpp"

namespace rtn {

// What a delivery statement of the generated code does (the host runs it when its bit is set).
enum class DeliverKind : uint32_t {
  Packet = 0,          // PacketContinue: `if let Some(p) = T::from_mbuf(mbuf) { cb(p, ..) }` (data.rs:306-317)
  TrackedPackets = 1,  // Packet layer, packet-level sub: drain `tracked.packets()` into cb (data.rs:318-330)
  Callback = 2,        // Packet layer, static/connection-level sub: build_callback (data.rs:332-393)
  Stream = 3,          // Packet layer, streaming sub: `tracked.streaming_<id>.matched()` (utils.rs:277-283)
};

// One callback invocation site in the generated code, in code (= execution) order.
struct DeliverStmt {
  uint32_t sub_id;       // subscription index in the spec
  bool payload;          // Payload datatype: fires only if the payload slice is readable
  std::string callback;  // callback name (for the host dispatcher)
  DeliverKind kind = DeliverKind::Packet;
};

// A condition of the PacketDeliver filter that depends on the connection, not the packet: a
// service test `matches!(conn.service(), ConnParser::X)` (utils.rs:459-486), or a session
// predicate looped over `tracked.sessions()` (deliver_filter.rs:123-151). The host supplies its
// value per connection: 0/1 for a service, the number of tracked sessions satisfying it for a
// session predicate (the body runs once per such session). One fact per distinct predicate.
struct PdFact {
  enum Kind : uint32_t { Service = 0, Session = 1 };
  Kind kind;
  std::string pred;      // the predicate as filter text
  std::string protocol;  // its protocol (the service / session type)
};

struct PdStmt {
  DeliverStmt d;
  std::vector<std::pair<uint32_t, uint32_t>> loops;  // enclosing session loops (tree node id, fact), outermost first
};

struct PacketProgram {
  std::vector<SubscriptionSpec> subs;
  PTree tree{FilterLayer::PacketContinue};
  std::vector<DeliverStmt> delivers;
  std::string hip_body;     // __device__ function rtn_filter(...) specialised to this tree (straight-line)
  std::string hip_body_branchy;  // the same as nested if/else (RTN_BRANCHY_FILTER experiment)
  std::string hip_body_chain;    // straight-line without range runs (RTN_CHAIN_FILTER experiment)
  std::string hip_body_fold;     // range runs + folded action flags (RTN_FOLD_ACT experiment)
  std::string rust_listing; // the Rust the reference filtergen would emit (normalised), for review
  bool wraps_ethernet = false;
  std::string hw_filter;    // get_hw_filter (filtergen/src/lib.rs:233-238): the NIC keep/drop filter
  uint32_t deliver_words() const { return (uint32_t)((delivers.size() + 63) / 64); }

  // first-packet filter (FilterLayer::Packet, the generated `packet_filter`, filtergen/src/lib.rs:284-285)
  PTree conn_tree{FilterLayer::Packet};
  std::vector<DeliverStmt> conn_delivers;
  std::string hip_conn_body;      // __device__ rtn_conn_filter(const rtn_cview&, data, term, cm)
  std::string rust_conn_listing;
  uint32_t conn_deliver_words() const { return (uint32_t)((conn_delivers.size() + 63) / 64); }

  // packet delivery for tracked connections (FilterLayer::PacketDeliver, the generated
  // `packet_deliver`, filtergen/src/lib.rs:299-304, 357-362)
  PTree pd_tree{FilterLayer::PacketDeliver};
  std::vector<PdStmt> pd_stmts;
  std::vector<PdFact> pd_facts;
  std::string hip_pd_body;   // __device__ rtn_pd_filter(const rtn_cview&, bool payload_ok, const rtn_u32* f, rtn_u32* cnt)
  std::string rust_pd_listing;
};

// Compile subscriptions into the PacketContinue program (and the first-packet filter). Throws FilterError on any filter
// the reference would reject at compile time (parse errors, layer errors, type errors).
PacketProgram compile_packet_program(const std::vector<SubscriptionSpec>& subs);

}  // namespace rtn
