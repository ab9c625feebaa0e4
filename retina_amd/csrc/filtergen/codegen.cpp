// PacketContinue code generation (see codegen.hpp for the reference map).
#include "codegen.hpp"

#include <cstdio>
#include <map>

namespace rtn {
namespace {

enum class FT { U8, U16, U32, BOOL, V4, V6 };

struct FieldDef {
  FT type;
  const char* hip;  // HIP expression over `v` (rtn_view) producing the accessor's value
};

// Public accessors of the packet parsers (core/src/protocols/packet/{ipv4,ipv6,tcp,udp}.rs) with
// their Rust return types. `rtn_l3_*` / `rtn_l4_*` read the fixed header views the kernel builds.
const std::map<std::string, FieldDef>& fields(const std::string& proto) {
  static const std::map<std::string, FieldDef> ipv4 = {
      {"version", {FT::U8, "((rtn_l3_b(v, 0) & 0xf0u) >> 4)"}},              // ipv4.rs:38-40
      {"ihl", {FT::U8, "(rtn_l3_b(v, 0) & 0x0fu)"}},                          // :44-46
      {"version_ihl", {FT::U8, "rtn_l3_b(v, 0)"}},                           // :50-52
      {"dscp", {FT::U8, "(rtn_l3_b(v, 1) >> 2)"}},                            // :56-58
      {"ecn", {FT::U8, "(rtn_l3_b(v, 1) & 0x03u)"}},                          // :62-64
      {"dscp_ecn", {FT::U8, "rtn_l3_b(v, 1)"}},                              // :68-70
      {"type_of_service", {FT::U8, "rtn_l3_b(v, 1)"}},                       // :74-76
      {"total_length", {FT::U16, "rtn_l3_be16(v, 2)"}},                      // :80-82
      {"identification", {FT::U16, "rtn_l3_be16(v, 4)"}},                    // :86-88
      {"flags_to_fragment_offset", {FT::U16, "rtn_l3_be16(v, 6)"}},          // :92-94
      {"flags", {FT::U8, "(rtn_l3_be16(v, 6) >> 13)"}},                       // :98-100
      {"rf", {FT::BOOL, "((rtn_l3_be16(v, 6) & 0x8000u) != 0u ? 1u : 0u)"}},  // :104-106
      {"df", {FT::BOOL, "((rtn_l3_be16(v, 6) & 0x4000u) != 0u ? 1u : 0u)"}},  // :110-112
      {"mf", {FT::BOOL, "((rtn_l3_be16(v, 6) & 0x2000u) != 0u ? 1u : 0u)"}},  // :116-118
      {"fragment_offset", {FT::U16, "(rtn_l3_be16(v, 6) & 0x1fffu)"}},        // :122-124
      {"time_to_live", {FT::U8, "rtn_l3_b(v, 8)"}},                          // :128-130
      {"protocol", {FT::U8, "rtn_l3_b(v, 9)"}},                              // :134-136
      {"header_checksum", {FT::U16, "rtn_l3_be16(v, 10)"}},                  // :140-142
      {"src_addr", {FT::V4, "rtn_l3_be32(v, 12)"}},                          // :146-148
      {"dst_addr", {FT::V4, "rtn_l3_be32(v, 16)"}},                          // :152-154
  };
  static const std::map<std::string, FieldDef> ipv6 = {
      {"version", {FT::U8, "((rtn_l3_be32(v, 0) & 0xf0000000u) >> 28)"}},    // ipv6.rs:31-34
      {"dscp", {FT::U8, "((rtn_l3_be32(v, 0) & 0x0fc00000u) >> 22)"}},       // :38-41
      {"ecn", {FT::U8, "((rtn_l3_be32(v, 0) & 0x00300000u) >> 20)"}},        // :45-48
      {"traffic_class", {FT::U8, "((rtn_l3_be32(v, 0) & 0x0ff00000u) >> 20)"}},  // :52-55
      {"flow_label", {FT::U32, "(rtn_l3_be32(v, 0) & 0x000fffffu)"}},         // :59-61
      {"version_to_flow_label", {FT::U32, "rtn_l3_be32(v, 0)"}},             // :65-67
      {"payload_length", {FT::U16, "rtn_l3_be16(v, 4)"}},                    // :71-73
      {"next_header", {FT::U8, "rtn_l3_b(v, 6)"}},                           // :77-79
      {"hop_limit", {FT::U8, "rtn_l3_b(v, 7)"}},                             // :83-85
      {"src_addr", {FT::V6, "8"}},                                            // :89-91 (byte offset)
      {"dst_addr", {FT::V6, "24"}},                                           // :95-97
  };
  static const std::map<std::string, FieldDef> tcp = {
      {"src_port", {FT::U16, "rtn_l4_be16(v, 0)"}},                          // tcp.rs:38-40
      {"dst_port", {FT::U16, "rtn_l4_be16(v, 2)"}},                          // :44-46
      {"seq_no", {FT::U32, "rtn_l4_be32(v, 4)"}},                            // :50-52
      {"ack_no", {FT::U32, "rtn_l4_be32(v, 8)"}},                            // :56-58
      {"data_offset", {FT::U8, "((rtn_l4_b(v, 12) & 0xf0u) >> 4)"}},          // :62-64
      {"reserved", {FT::U8, "(rtn_l4_b(v, 12) & 0x0fu)"}},                    // :68-70
      {"data_offset_to_ns", {FT::U8, "rtn_l4_b(v, 12)"}},                    // :74-76
      {"flags", {FT::U8, "rtn_l4_b(v, 13)"}},                                // :80-82
      {"window", {FT::U16, "rtn_l4_be16(v, 14)"}},                           // :86-88
      {"checksum", {FT::U16, "rtn_l4_be16(v, 16)"}},                         // :92-94
      {"urgent_pointer", {FT::U16, "rtn_l4_be16(v, 18)"}},                   // :98-100
      {"ns", {FT::U8, "(rtn_l4_b(v, 12) & 0x01u)"}},                          // :106-108
      {"cwr", {FT::U8, "((rtn_l4_b(v, 13) >> 7) & 1u)"}},                     // :112-114
      {"ece", {FT::U8, "((rtn_l4_b(v, 13) >> 6) & 1u)"}},                     // :118-120
      {"urg", {FT::U8, "((rtn_l4_b(v, 13) >> 5) & 1u)"}},                     // :124-126
      {"ack", {FT::U8, "((rtn_l4_b(v, 13) >> 4) & 1u)"}},                     // :130-132
      {"psh", {FT::U8, "((rtn_l4_b(v, 13) >> 3) & 1u)"}},                     // :136-138
      {"rst", {FT::U8, "((rtn_l4_b(v, 13) >> 2) & 1u)"}},                     // :142-144
      {"syn", {FT::U8, "((rtn_l4_b(v, 13) >> 1) & 1u)"}},                     // :148-150
      {"fin", {FT::U8, "(rtn_l4_b(v, 13) & 1u)"}},                            // :154-156
      {"synack", {FT::U8, "((rtn_l4_b(v, 13) & 0x12u) != 0u ? 1u : 0u)"}},    // :160-162 (SYN or ACK)
  };
  static const std::map<std::string, FieldDef> udp = {
      {"src_port", {FT::U16, "rtn_l4_be16(v, 0)"}},                          // udp.rs:24-26
      {"dst_port", {FT::U16, "rtn_l4_be16(v, 2)"}},                          // :30-32
      {"length", {FT::U16, "rtn_l4_be16(v, 4)"}},                            // :36-38
      {"checksum", {FT::U16, "rtn_l4_be16(v, 6)"}},                          // :42-44
  };
  static const std::map<std::string, FieldDef> none;
  if (proto == "ipv4") return ipv4;
  if (proto == "ipv6") return ipv6;
  if (proto == "tcp") return tcp;
  if (proto == "udp") return udp;
  return none;
}

// The first-packet filter (FilterLayer::Packet) may only test connection-invariant fields: the
// tree build rejects every other one (Predicate::req_packet, ast.rs:118-133; ptree.rs:406-415),
// and those all live in the forwarded frame's L4Context. `c` is the kernel's rtn_cview.
const std::map<std::string, FieldDef>& conn_fields(const std::string& proto) {
  static const std::map<std::string, FieldDef> ipv4 = {{"src_addr", {FT::V4, "c.src4"}}, {"dst_addr", {FT::V4, "c.dst4"}}};
  static const std::map<std::string, FieldDef> ipv6 = {{"src_addr", {FT::V6, "c.s6"}}, {"dst_addr", {FT::V6, "c.d6"}}};
  static const std::map<std::string, FieldDef> l4 = {{"src_port", {FT::U16, "c.sport"}}, {"dst_port", {FT::U16, "c.dport"}}};
  static const std::map<std::string, FieldDef> none;
  if (proto == "ipv4") return ipv4;
  if (proto == "ipv6") return ipv6;
  if (proto == "tcp" || proto == "udp") return l4;
  return none;
}

const char* camel(const std::string& p) {
  if (p == "ethernet") return "Ethernet";
  if (p == "ipv4") return "Ipv4";
  if (p == "ipv6") return "Ipv6";
  if (p == "tcp") return "Tcp";
  if (p == "udp") return "Udp";
  return "?";
}

uint64_t type_max(FT t) {
  switch (t) {
    case FT::U8: return 0xff;
    case FT::U16: return 0xffff;
    case FT::U32: return 0xffffffffull;
    default: return 0;
  }
}

bool is_int(FT t) { return t == FT::U8 || t == FT::U16 || t == FT::U32; }

// HIP literal of a predicate constant, wrapped in RTN_K (pc_kernel.hip: the identity unless a
// timing variant redefines it)
std::string u32lit(uint64_t v) { return "RTN_K(" + std::to_string(v) + "u)"; }

struct Gen {
  PacketProgram& prog;
  std::string hip, rust;
  FilterLayer layer = FilterLayer::PacketContinue;
  bool range_runs = true;  // pc_flat lowers range runs (RangeRun)

  [[noreturn]] void type_error(const Predicate& p, const std::string& why) {
    throw FilterError("filter does not type-check (" + p.str() + "): " + why);
  }

  // binary_to_tokens (utils.rs:18-249): returns {hip_expr, rust_expr}
  std::pair<std::string, std::string> binary(const Predicate& p) {
    const bool conn = layer == FilterLayer::Packet || layer == FilterLayer::PacketDeliver;
    const auto& tab = conn ? conn_fields(p.protocol) : fields(p.protocol);
    auto it = tab.find(p.field);
    if (it == tab.end()) {
      if (conn) throw FilterError("internal: per-packet field " + p.str() + " after the packet filter");
      type_error(p, "no method named `" + p.field + "` on `" + camel(p.protocol) + "`");
    }
    const FieldDef& fd = it->second;
    const std::string racc = p.protocol + "." + p.field + "()";
    const Value& val = p.value;
    auto bad_op = [&]() { type_error(p, std::string("Invalid binary operation `") + binop_str(p.op) + "` for value"); };
    switch (val.kind) {
      case VKind::Int: {
        const char* op = nullptr;
        switch (p.op) {
          case BinOp::Eq: op = "=="; break;
          case BinOp::Ne: op = "!="; break;
          case BinOp::Ge: op = ">="; break;
          case BinOp::Le: op = "<="; break;
          case BinOp::Gt: op = ">"; break;
          case BinOp::Lt: op = "<"; break;
          default: bad_op();
        }
        if (!is_int(fd.type)) type_error(p, "mismatched types: integer literal against a non-integer accessor");
        if (val.i > type_max(fd.type)) type_error(p, "literal out of range for the accessor's type");
        return {"(" + std::string(fd.hip) + " " + op + " " + u32lit(val.i) + ")",
                racc + " " + op + " " + std::to_string(val.i)};
      }
      case VKind::IntRange: {
        if (p.op != BinOp::In) bad_op();
        if (!is_int(fd.type)) type_error(p, "mismatched types: integer literal against a non-integer accessor");
        if (val.to > type_max(fd.type) || val.i > type_max(fd.type))
          type_error(p, "literal out of range for the accessor's type");
        return {"((" + std::string(fd.hip) + " >= " + u32lit(val.i) + ") && (" + fd.hip + " <= " + u32lit(val.to) + "))",
                racc + " >= " + std::to_string(val.i) + " && " + racc + " <= " + std::to_string(val.to)};
      }
      case VKind::Ipv4: {
        if (p.op != BinOp::Eq && p.op != BinOp::Ne && p.op != BinOp::In) bad_op();
        if (fd.type == FT::V6) type_error(p, "the trait `From<Ipv6Addr>` is not implemented for `u32`");
        uint32_t addr = val.v4.addr, mask = val.v4.netmask(), net = addr & mask;
        bool ne = p.op == BinOp::Ne;
        std::string x = fd.hip;
        std::string rx = "u32::from(" + racc + ")";
        if (val.v4.prefix == 32)
          return {"(" + x + (ne ? " != " : " == ") + u32lit(addr) + ")",
                  rx + (ne ? " != " : " == ") + std::to_string(addr)};
        return {"((" + x + " & " + u32lit(mask) + ")" + (ne ? " != " : " == ") + u32lit(net) + ")",
                rx + " & " + std::to_string(mask) + (ne ? " != " : " == ") + std::to_string(net)};
      }
      case VKind::Ipv6: {
        if (p.op != BinOp::Eq && p.op != BinOp::Ne && p.op != BinOp::In) bad_op();
        if (fd.type == FT::V4) type_error(p, "the trait `From<Ipv4Addr>` is not implemented for `u128`");
        U128 addr = val.v6.addr, mask = val.v6.netmask(), net = addr & mask;
        bool full = val.v6.prefix == 128;
        bool ne = p.op == BinOp::Ne;
        uint32_t aw[4] = {(uint32_t)(addr.hi >> 32), (uint32_t)addr.hi, (uint32_t)(addr.lo >> 32), (uint32_t)addr.lo};
        uint32_t mw[4] = {(uint32_t)(mask.hi >> 32), (uint32_t)mask.hi, (uint32_t)(mask.lo >> 32), (uint32_t)mask.lo};
        uint32_t nw[4] = {(uint32_t)(net.hi >> 32), (uint32_t)net.hi, (uint32_t)(net.lo >> 32), (uint32_t)net.lo};
        std::string conj;
        for (int k = 0; k < 4; ++k) {
          std::string word;
          if (fd.type == FT::V6 && conn) word = std::string(fd.hip) + "[" + std::to_string(k) + "]";
          else if (fd.type == FT::V6) word = "rtn_l3_be32(v, " + std::string(fd.hip) + " + " + std::to_string(4 * k) + ")";
          else word = k == 3 ? std::string(fd.hip) : std::string("0u");
          std::string term = full ? "(" + word + " == " + u32lit(aw[k]) + ")"
                                  : "((" + word + " & " + u32lit(mw[k]) + ") == " + u32lit(nw[k]) + ")";
          conj += (k ? " && " : "") + term;
        }
        std::string rx = "u128::from(" + racc + ")";
        std::string hexpr = ne ? "(!(" + conj + "))" : "(" + conj + ")";
        if (full) return {hexpr, rx + (ne ? " != " : " == ") + addr.to_dec()};
        return {hexpr, rx + " & " + mask.to_dec() + (ne ? " != " : " == ") + net.to_dec()};
      }
      case VKind::Text:
        type_error(p, "string values cannot be compared with packet header accessors");
      case VKind::Byte:
        type_error(p, "byte values cannot be compared with packet header accessors");
    }
    type_error(p, "unsupported value");
  }

  static std::string ind(int d) { return std::string(2 * d, ' '); }

  // update_body (utils.rs:251-285)
  void update_body(const PNode& n, int d) {
    if (layer == FilterLayer::Packet) {
      update_body_conn(n, d);
      return;
    }
    if (!n.actions.drop()) {
      hip += ind(d) + "act |= " + u32lit(n.actions.data) + ";\n";
      rust += ind(d) + "result.push(Actions{data:" + std::to_string(n.actions.data) + ",terminal:" +
              std::to_string(n.actions.terminal) + "});\n";
    }
    for (auto& dv : n.deliver) {
      const SubscriptionSpec& spec = prog.subs.at(dv.id);
      if (spec.level != Level::Packet) throw FilterError("internal: non-packet delivery at PacketContinue");
      // build_packet_callback (data.rs:299-331) / build_packet_params (data.rs:262-297)
      std::string ty, params;
      for (auto& dt : spec.datatypes) {
        if (!params.empty()) params += ", ";
        if (dt.level == Level::Packet) {
          ty = dt.as_str;
          params += "p";
        } else if (dt.as_str == "FilterStr") {
          params += "&\"" + spec.filter + "\"";
        } else if (dt.as_str == "CoreId") {
          params += "core_id";
        } else {
          throw FilterError("Invalid datatype in packet callback: " + dt.as_str);
        }
      }
      if (ty != "ZcFrame" && ty != "Payload") throw FilterError("unsupported packet datatype " + ty);
      uint32_t k = (uint32_t)prog.delivers.size();
      prog.delivers.push_back(DeliverStmt{(uint32_t)dv.id, ty == "Payload", spec.callback, DeliverKind::Packet});
      std::string bit = "dm[" + std::to_string(k / 64) + "] |= (1ull << " + std::to_string(k % 64) + ");";
      if (ty == "Payload") hip += ind(d) + "if (v.payload_ok) { " + bit + " }\n";
      else hip += ind(d) + bit + "\n";
      rust += ind(d) + "if let Some(p) = " + ty + "::from_mbuf(mbuf) { " + spec.callback + "(" + params + "); }\n";
    }
  }

  // update_body at FilterLayer::Packet: actions with their terminal half, then the statements
  // the host runs with its tracked data (build_packet_callback's tracked-packet drain,
  // data.rs:318-330; build_callback, data.rs:332-393; streaming `matched()`, utils.rs:277-283)
  // recorded as statement-mask bits in code order.
  void update_body_conn(const PNode& n, int d) {
    if (!n.actions.drop()) {
      hip += ind(d) + "data |= " + u32lit(n.actions.data) + "; term |= " + u32lit(n.actions.terminal) + ";\n";
      rust += ind(d) + "result.push(Actions{data:" + std::to_string(n.actions.data) + ",terminal:" +
              std::to_string(n.actions.terminal) + "});\n";
    }
    auto stmt = [&](uint32_t sub, DeliverKind kind, const std::string& rust_stmt) {
      uint32_t k = (uint32_t)prog.conn_delivers.size();
      prog.conn_delivers.push_back(DeliverStmt{sub, false, prog.subs.at(sub).callback, kind});
      hip += ind(d) + "cm[" + std::to_string(k / 64) + "] |= (1ull << " + std::to_string(k % 64) + ");\n";
      rust += ind(d) + rust_stmt + "\n";
    };
    for (auto& dv : n.deliver) {
      const SubscriptionSpec& spec = prog.subs.at(dv.id);
      if (spec.level == Level::Packet)
        stmt((uint32_t)dv.id, DeliverKind::TrackedPackets,
             "for mbuf in tracked.packets() { /* " + spec.callback + " */ }");
      else
        stmt((uint32_t)dv.id, DeliverKind::Callback, spec.callback + "(/* tracked */);");
    }
    for (auto& sv : n.stream)
      stmt((uint32_t)sv.id, DeliverKind::Stream, "tracked.streaming_" + std::to_string(sv.id) + ".matched();");
  }

  // gen_packet_filter_util (packet_filter.rs:31-73)
  void children(const PNode& n, int d) {
    bool first_unary = true;
    for (auto& c : n.children) {
      if (!c.pred.on_packet()) continue;
      if (c.pred.is_unary()) {
        const std::string& proto = c.pred.protocol;
        std::string cond;
        const char* vv = layer == FilterLayer::Packet ? "c." : "v.";
        if (proto == "ipv4") cond = std::string(vv) + "v4";
        else if (proto == "ipv6") cond = std::string(vv) + "v6";
        else if (proto == "tcp") cond = std::string(vv) + "tcp";
        else if (proto == "udp") cond = std::string(vv) + "udp";
        else throw FilterError("internal: unexpected packet protocol " + proto);
        hip += ind(d) + (first_unary ? "if (" : "else if (") + cond + ") {\n";
        rust += ind(d) + (first_unary ? "if let Ok(" : "else if let Ok(") + proto + ") = parse_to::<" + camel(proto) +
                ">(" + n.pred.protocol + ") {\n";
        first_unary = false;
      } else {
        auto ex = binary(c.pred);
        hip += ind(d) + (c.if_else ? "else if " : "if ") + ex.first + " {\n";
        rust += ind(d) + (c.if_else ? "else if " : "if ") + ex.second + " {\n";
      }
      children(c, d + 1);
      update_body(c, d + 1);
      hip += ind(d) + "}\n";
      rust += ind(d) + "}\n";
    }
  }


  // ---- PacketContinue as straight-line HIP (the default body): every node's reach flag is a
  // select chain, actions and delivery bits are OR-ed in under their node's flag. A wave whose
  // lanes take different branches runs all of them anyway; this form drops the exec-mask
  // bookkeeping of each branch. Statement numbering follows children() / update_body().
  uint32_t flat_pc_stmt = 0;
  // Actions folded into one flag per distinct action word, OR-ed over the reach flags of the
  // nodes that carry it, and `act |= flag ? word : 0` once per word at the end (the
  // RTN_FOLD_ACT experiment; the product form ORs each node's word under its flag).
  bool fold_act = false;
  std::map<uint32_t, std::string> act_flags{};
  void act_or(const PNode& n, const std::string& R) {
    if (n.actions.drop()) return;
    if (!fold_act) {
      hip += "  act |= " + R + " ? " + u32lit(n.actions.data) + " : 0u;\n";
      return;
    }
    auto it = act_flags.find(n.actions.data);
    if (it == act_flags.end())
      it = act_flags.emplace(n.actions.data, "a" + std::to_string(act_flags.size())).first;
    hip += "  " + it->second + " = " + it->second + " || " + R + ";\n";
  }
  std::string act_prologue() const {
    std::string s;
    for (auto& kv : act_flags) s += "  bool " + kv.second + " = false;\n";
    return s;
  }
  std::string act_epilogue() const {
    std::string s;
    for (auto& kv : act_flags) s += "  act |= " + kv.second + " ? " + u32lit(kv.first) + " : 0u;\n";
    return s;
  }
  void pc_flat_body(const PNode& n, const std::string& R) {
    act_or(n, R);
    for (auto& dv : n.deliver) {
      uint32_t k = flat_pc_stmt++;
      if (k >= prog.delivers.size() || prog.delivers[k].sub_id != (uint32_t)dv.id)
        throw FilterError("internal: packet-continue statement order");
      std::string reach = prog.delivers[k].payload ? "(" + R + " && v.payload_ok)" : R;
      hip += "  RTN_DM_SET(dm, " + std::to_string(k / 64) + ", " + std::to_string(k % 64) + ", " + reach + ");\n";
    }
  }
  // A run of sibling leaves that test one header field for equality against constants in
  // arithmetic progression (`ipv4.dst_addr = 10.k.0.0/16` for k = 0..18; ports 80, 81, 82, ...),
  // each delivering one packet-level statement with consecutive statement numbers and the same
  // actions. The tests are mutually exclusive, so the run is one subtract-and-compare: the lane's
  // offset into the progression picks its statement bit. The reach flags, the chain flag T and the
  // statement bits come out as the per-child chain would produce them (pc_flat below).
  struct RangeRun {
    size_t len = 0;      // children in the run (0: no run here)
    std::string x;       // the field (masked) as a u32 expression
    uint64_t c0 = 0;     // its value at the run's first child
    unsigned shift = 0;  // log2 of the progression's step
  };
  static constexpr size_t kRangeRunMin = 4;
  bool range_key(const Predicate& p, std::string& x, uint64_t& c, unsigned& shift) const {
    if (!p.is_binary() || !p.on_packet() || p.op != BinOp::Eq) return false;
    const auto& tab = fields(p.protocol);
    auto it = tab.find(p.field);
    if (it == tab.end()) return false;
    const FieldDef& fd = it->second;
    if (p.value.kind == VKind::Int && is_int(fd.type) && p.value.i <= type_max(fd.type)) {
      x = fd.hip, c = p.value.i, shift = 0;
      return true;
    }
    if (p.value.kind == VKind::Ipv4 && fd.type == FT::V4 && p.value.v4.prefix >= 1) {
      uint32_t mask = p.value.v4.netmask();
      x = p.value.v4.prefix == 32 ? std::string(fd.hip) : "(" + std::string(fd.hip) + " & " + u32lit(mask) + ")";
      c = p.value.v4.addr & mask, shift = 32 - p.value.v4.prefix;
      return true;
    }
    return false;
  }
  RangeRun range_run(const PNode& n, size_t i, size_t stmt0) const {
    RangeRun run;
    const auto& ch = n.children;
    auto leaf_one_stmt = [&](const PNode& c) {
      for (auto& g : c.children)
        if (g.pred.on_packet()) return false;
      return c.deliver.size() == 1 && c.stream.empty();
    };
    std::string x0;
    uint64_t c0;
    unsigned s0;
    if (!range_key(ch[i].pred, x0, c0, s0) || !leaf_one_stmt(ch[i])) return run;
    const bool payload = stmt0 < prog.delivers.size() && prog.delivers[stmt0].payload;
    size_t len = 1;
    for (size_t j = i + 1; j < ch.size(); ++j, ++len) {
      const PNode& c = ch[j];
      std::string x;
      uint64_t cv;
      unsigned s;
      if (!c.if_else || !range_key(c.pred, x, cv, s) || x != x0 || s != s0) break;
      if (cv != c0 + (uint64_t(len) << s0) || !leaf_one_stmt(c) || !(c.actions == ch[i].actions)) break;
      const size_t k = stmt0 + len;
      if (k >= prog.delivers.size() || prog.delivers[k].payload != payload || (stmt0 % 64) + len >= 64) break;
      if (prog.delivers[k].sub_id != (uint32_t)c.deliver.begin()->id) break;
    }
    if (len < kRangeRunMin) return run;
    run.len = len, run.x = x0, run.c0 = c0, run.shift = s0;
    return run;
  }
  void pc_flat_range(const PNode& n, size_t i, const RangeRun& run, const std::string& R, std::string& T,
                     bool is_else) {
    const PNode& first = n.children[i];
    const std::string id = std::to_string(first.id);
    const uint32_t k0 = flat_pc_stmt;
    for (size_t j = 0; j < run.len; ++j) {
      const uint32_t k = flat_pc_stmt++;
      if (k >= prog.delivers.size() || prog.delivers[k].sub_id != (uint32_t)n.children[i + j].deliver.begin()->id)
        throw FilterError("internal: packet-continue statement order");
    }
    const uint64_t span = uint64_t(run.len) << run.shift;  // <= 2^32: the keys are distinct u32 values
    hip += "  const rtn_u32 q" + id + " = " + run.x + " - " + u32lit(run.c0) + ";\n";
    hip += "  const bool k" + id + " = (unsigned long long)q" + id + " < " + std::to_string(span) + "ull;\n";
    const std::string rc = "r" + id;
    if (!is_else || T.empty()) {
      T = "t" + id;
      hip += "  bool " + T + " = k" + id + ";\n";
      hip += "  const bool " + rc + " = " + R + " && k" + id + ";\n";
    } else {
      hip += "  const bool " + rc + " = " + R + " && !" + T + " && k" + id + ";\n";
      hip += "  " + T + " = " + T + " || k" + id + ";\n";
    }
    act_or(first, rc);
    const std::string reach = prog.delivers[k0].payload ? "(" + rc + " && v.payload_ok)" : rc;
    hip += "  RTN_DM_SETV(dm, " + std::to_string(k0 / 64) + ", " + std::to_string(k0 % 64) + " + (q" + id + " >> " +
           std::to_string(run.shift) + "), " + reach + ");\n";
  }

  void pc_flat(const PNode& n, const std::string& R) {
    bool first_unary = true;
    std::string T;
    for (size_t ci = 0; ci < n.children.size(); ++ci) {
      const PNode& c = n.children[ci];
      if (!c.pred.on_packet()) continue;
      if (range_runs && c.pred.is_binary()) {
        const RangeRun run = range_run(n, ci, flat_pc_stmt);
        if (run.len) {
          pc_flat_range(n, ci, run, R, T, c.if_else);
          ci += run.len - 1;
          continue;
        }
      }
      const std::string id = std::to_string(c.id);
      std::string cond;
      bool is_else;
      if (c.pred.is_unary()) {
        const std::string& proto = c.pred.protocol;
        cond = proto == "ipv4" ? "v.v4" : proto == "ipv6" ? "v.v6" : proto == "tcp" ? "v.tcp" : "v.udp";
        is_else = !first_unary;
        first_unary = false;
      } else {
        cond = binary(c.pred).first;
        is_else = c.if_else;
      }
      const std::string rc = "r" + id;
      hip += "  const bool k" + id + " = " + cond + ";\n";
      if (!is_else || T.empty()) {
        T = "t" + id;
        hip += "  bool " + T + " = k" + id + ";\n";
        hip += "  const bool " + rc + " = " + R + " && k" + id + ";\n";
      } else {
        hip += "  const bool " + rc + " = " + R + " && !" + T + " && k" + id + ";\n";
        hip += "  " + T + " = " + T + " || k" + id + ";\n";
      }
      pc_flat(c, rc);
      pc_flat_body(c, rc);
    }
  }


  // ---- FilterLayer::Packet (packet_filter) as straight-line HIP, like pc_flat: actions with
  // their terminal half and statement-mask bits under each node's reach flag. Statement
  // numbering follows children() / update_body_conn().
  uint32_t flat_conn_stmt = 0;
  void conn_flat_body(const PNode& n, const std::string& R) {
    if (!n.actions.drop())
      hip += "  data |= " + R + " ? " + u32lit(n.actions.data) + " : 0u; term |= " + R + " ? " +
             u32lit(n.actions.terminal) + " : 0u;\n";
    auto stmt = [&](uint32_t sub) {
      uint32_t k = flat_conn_stmt++;
      if (k >= prog.conn_delivers.size() || prog.conn_delivers[k].sub_id != sub)
        throw FilterError("internal: packet-filter statement order");
      hip += "  RTN_DM_SET(cm, " + std::to_string(k / 64) + ", " + std::to_string(k % 64) + ", " + R + ");\n";
    };
    for (auto& dv : n.deliver) stmt((uint32_t)dv.id);
    for (auto& sv : n.stream) stmt((uint32_t)sv.id);
  }
  void conn_flat(const PNode& n, const std::string& R) {
    bool first_unary = true;
    std::string T;
    for (auto& c : n.children) {
      if (!c.pred.on_packet()) continue;
      const std::string id = std::to_string(c.id);
      std::string cond;
      bool is_else;
      if (c.pred.is_unary()) {
        const std::string& proto = c.pred.protocol;
        cond = proto == "ipv4" ? "c.v4" : proto == "ipv6" ? "c.v6" : proto == "tcp" ? "c.tcp" : "c.udp";
        is_else = !first_unary;
        first_unary = false;
      } else {
        cond = binary(c.pred).first;
        is_else = c.if_else;
      }
      const std::string rc = "r" + id;
      hip += "  const bool k" + id + " = " + cond + ";\n";
      if (!is_else || T.empty()) {
        T = "t" + id;
        hip += "  bool " + T + " = k" + id + ";\n";
        hip += "  const bool " + rc + " = " + R + " && k" + id + ";\n";
      } else {
        hip += "  const bool " + rc + " = " + R + " && !" + T + " && k" + id + ";\n";
        hip += "  " + T + " = " + T + " || k" + id + ";\n";
      }
      conn_flat(c, rc);
      conn_flat_body(c, rc);
    }
  }

  // ---- FilterLayer::PacketDeliver (deliver_filter.rs) ----
  // The body multiplies `m` (how many times the enclosing session loops run it) into per-statement
  // counts; `f` holds the connection's facts (PdFact) and `pok` the Payload guard.

  uint32_t pd_fact(const PNode& c, PdFact::Kind kind) {
    const std::string text = c.pred.str();
    for (size_t k = 0; k < prog.pd_facts.size(); ++k)
      if (prog.pd_facts[k].kind == kind && prog.pd_facts[k].pred == text) return (uint32_t)k;
    prog.pd_facts.push_back(PdFact{kind, text, c.pred.protocol});
    return (uint32_t)prog.pd_facts.size() - 1u;
  }

  // update_body (utils.rs:251-285) at PacketDeliver: no actions (with_term_filter and
  // with_nonterm_filter are empty there, datatypes.rs:704-721); build_packet_callback for each
  // delivery (data.rs:299-317: `if let Some(p) = T::from_mbuf(mbuf) { cb(p, ..) }`).
  void pd_update_body(const PNode& n, int d, const std::string& m, const std::vector<std::pair<uint32_t, uint32_t>>& loops) {
    if (!n.actions.drop()) throw FilterError("internal: actions in the packet-deliver filter");
    if (!n.stream.empty()) throw FilterError("internal: streaming delivery in the packet-deliver filter");
    for (auto& dv : n.deliver) {
      const SubscriptionSpec& spec = prog.subs.at(dv.id);
      if (spec.level != Level::Packet) throw FilterError("internal: non-packet delivery in the packet-deliver filter");
      std::string ty, params;
      for (auto& dt : spec.datatypes) {
        if (!params.empty()) params += ", ";
        if (dt.level == Level::Packet) {
          ty = dt.as_str;
          params += "p";
        } else if (dt.as_str == "FilterStr") {
          params += "&\"" + spec.filter + "\"";
        } else if (dt.as_str == "CoreId") {
          params += "tracked.core_id()";  // data.rs:285-292: from the tracked data after PacketContinue
        } else {
          throw FilterError("Invalid datatype in packet callback: " + dt.as_str);
        }
      }
      if (ty != "ZcFrame" && ty != "Payload") throw FilterError("unsupported packet datatype " + ty);
      uint32_t k = (uint32_t)prog.pd_stmts.size();
      prog.pd_stmts.push_back(PdStmt{DeliverStmt{(uint32_t)dv.id, ty == "Payload", spec.callback, DeliverKind::Packet}, loops});
      std::string add = "cnt[" + std::to_string(k) + "] += " + m + ";";
      hip += ind(d) + (ty == "Payload" ? "if (pok) { " + add + " }" : add) + "\n";
      rust += ind(d) + "if let Some(p) = " + ty + "::from_mbuf(mbuf) { " + spec.callback + "(" + params + "); }\n";
    }
  }

  // gen_deliver_util (deliver_filter.rs:31-121) with PacketDataFilter for packet predicates
  // (utils.rs:298-361), ConnDataFilter::add_service_pred (utils.rs:459-486) and add_session_pred
  // (deliver_filter.rs:123-151).
  void pd_children(const PNode& n, int d, const std::string& m, const std::vector<std::pair<uint32_t, uint32_t>>& loops) {
    bool first_unary = true, prev_loop = false;
    // an `else` right after a session loop is not Rust: filtergen's output would not compile
    auto no_else_after_loop = [&](bool is_else, const PNode& c) {
      if (is_else && prev_loop)
        throw FilterError("the generated packet_deliver does not compile: `else` after a session loop at " + c.pred.str());
    };
    for (auto& c : n.children) {
      std::string cm = m;
      std::vector<std::pair<uint32_t, uint32_t>> cl = loops;
      int closes = 1;
      if (c.pred.is_unary()) {
        const std::string& proto = c.pred.protocol;
        if (c.pred.on_packet()) {
          std::string cond;
          if (proto == "ipv4") cond = "c.v4";
          else if (proto == "ipv6") cond = "c.v6";
          else if (proto == "tcp") cond = "c.tcp";
          else if (proto == "udp") cond = "c.udp";
          else throw FilterError("internal: unexpected packet protocol " + proto);
          no_else_after_loop(!first_unary, c);
          hip += ind(d) + (first_unary ? "if (" : "else if (") + cond + ") {\n";
          rust += ind(d) + (first_unary ? "if let Ok(" : "else if let Ok(") + proto + ") = parse_to::<" + camel(proto) +
                  ">(" + n.pred.protocol + ") {\n";
          first_unary = false;
        } else if (c.pred.on_proto()) {
          no_else_after_loop(c.if_else, c);
          uint32_t k = pd_fact(c, PdFact::Service);
          hip += ind(d) + (c.if_else ? "else if (f[" : "if (f[") + std::to_string(k) + "] != 0u) {\n";
          std::string svc = proto;
          if (!svc.empty()) svc[0] = (char)toupper(svc[0]);
          rust += ind(d) + (c.if_else ? "else if " : "if ") + "matches!(conn.service(), ConnParser::" + svc + " { .. }) {\n";
        } else {
          throw FilterError("Unary predicate on session filter");
        }
      } else if (c.pred.on_packet()) {
        no_else_after_loop(c.if_else, c);
        auto ex = binary(c.pred);
        hip += ind(d) + (c.if_else ? "else if " : "if ") + ex.first + " {\n";
        rust += ind(d) + (c.if_else ? "else if " : "if ") + ex.second + " {\n";
      } else if (c.pred.on_session()) {
        uint32_t k = pd_fact(c, PdFact::Session);
        cm = "m" + std::to_string(d);
        cl.push_back({(uint32_t)c.id, k});
        hip += ind(d) + "{\n" + ind(d + 1) + "const rtn_u32 " + cm + " = " + m + " * f[" + std::to_string(k) + "];\n" +
               ind(d + 1) + "if (" + cm + " != 0u) {\n";
        std::string svc = c.pred.protocol;
        if (!svc.empty()) svc[0] = (char)toupper(svc[0]);
        rust += ind(d) + "for session in tracked.sessions() {\n" + ind(d + 1) + "if let SessionData::" + svc + "(" +
                c.pred.protocol + ") = &session.data {\n" + ind(d + 2) + "if /* " + c.pred.str() + " */ {\n";
        closes = 2;
        d += 1;
      } else {
        throw FilterError("Binary predicate on protocol filter");
      }
      prev_loop = closes == 2;
      pd_children(c, d + 1, cm, cl);
      pd_update_body(c, d + 1, cm, cl);
      if (closes == 2) {
        hip += ind(d) + "}\n" + ind(d - 1) + "}\n";
        rust += ind(d + 1) + "}\n" + ind(d) + "}\n" + ind(d - 1) + "}\n";
        d -= 1;
      } else {
        hip += ind(d) + "}\n";
        rust += ind(d) + "}\n";
      }
    }
  }
  // The same tree as straight-line HIP: every node's reach flag and multiplier is computed with
  // selects, and each statement's count is assigned once. (Branchy code let the compiler sink the
  // `cnt[k] += m` of sibling branches into one store with a computed index, which moves the
  // counters to scratch memory.) Statement and fact numbering follow pd_children / pd_update_body.
  uint32_t flat_stmt = 0;
  void pd_flat_body(const PNode& n, const std::string& R, const std::string& M) {
    for (auto& dv : n.deliver) {
      uint32_t k = flat_stmt++;
      if (k >= prog.pd_stmts.size() || prog.pd_stmts[k].d.sub_id != (uint32_t)dv.id)
        throw FilterError("internal: packet-deliver statement order");
      std::string reach = prog.pd_stmts[k].d.payload ? "(" + R + " && pok)" : R;
      hip += "  cnt[" + std::to_string(k) + "] = " + reach + " ? " + M + " : 0u;\n";
    }
  }
  void pd_flat(const PNode& n, const std::string& R, const std::string& M) {
    bool first_unary = true;
    std::string T;  // the open if-chain's "some branch taken" flag
    for (auto& c : n.children) {
      const std::string id = std::to_string(c.id);
      std::string rc = "r" + id, mc = M;
      if (!c.pred.is_unary() && c.pred.on_session()) {
        uint32_t k = pd_fact(c, PdFact::Session);
        mc = "m" + id;
        hip += "  const rtn_u32 " + mc + " = " + M + " * f[" + std::to_string(k) + "];\n";
        hip += "  const bool " + rc + " = " + R + " && " + mc + " != 0u;\n";
        T.clear();
      } else {
        std::string cond;
        bool is_else;
        if (c.pred.is_unary() && c.pred.on_packet()) {
          const std::string& proto = c.pred.protocol;
          cond = proto == "ipv4" ? "c.v4" : proto == "ipv6" ? "c.v6" : proto == "tcp" ? "c.tcp" : "c.udp";
          is_else = !first_unary;
          first_unary = false;
        } else if (c.pred.is_unary()) {
          cond = "(f[" + std::to_string(pd_fact(c, PdFact::Service)) + "] != 0u)";
          is_else = c.if_else;
        } else {
          cond = binary(c.pred).first;
          is_else = c.if_else;
        }
        hip += "  const bool k" + id + " = " + cond + ";\n";
        if (!is_else || T.empty()) {
          T = "t" + id;
          hip += "  bool " + T + " = k" + id + ";\n";
          hip += "  const bool " + rc + " = " + R + " && k" + id + ";\n";
        } else {
          hip += "  const bool " + rc + " = " + R + " && !" + T + " && k" + id + ";\n";
          hip += "  " + T + " = " + T + " || k" + id + ";\n";
        }
      }
      pd_flat(c, rc, mc);
      pd_flat_body(c, rc, mc);
    }
  }
};

}  // namespace

// Trees up to this many nodes are emitted straight-line (cfg4's 127-node tree: -8 % kernel time).
constexpr size_t kFlatMaxNodes = 256;

PacketProgram compile_packet_program(const std::vector<SubscriptionSpec>& subs) {
  PacketProgram prog;
  prog.subs = subs;
  for (auto& s : prog.subs) s.validate_spec();
  // filtergen builds every layer's tree (filtergen/src/lib.rs:274-304) and rejects the program
  // if any of them panics (e.g. a per-packet field in a connection-level filter, ptree.rs:406-415)
  for (FilterLayer l : {FilterLayer::Protocol, FilterLayer::Session, FilterLayer::ConnectionDeliver})
    (void)filter_subtree(l, prog.subs);
  prog.pd_tree = filter_subtree(FilterLayer::PacketDeliver, prog.subs);
  prog.tree = filter_subtree(FilterLayer::PacketContinue, prog.subs);
  prog.conn_tree = filter_subtree(FilterLayer::Packet, prog.subs);
  // get_hw_filter (filtergen/src/lib.rs:233-238): the PacketContinue tree's paths as one filter
  // string, which filtergen re-parses and panics on if invalid ("Invalid HW filter")
  prog.hw_filter = prog.tree.to_filter_string();
  try {
    (void)Filter::make(prog.hw_filter);
  } catch (const FilterError& e) {
    throw FilterError("Invalid HW filter " + prog.hw_filter + ": " + e.what());
  }
  const PNode& root = prog.tree.root;
  if (root.actions.terminal != 0) throw FilterError("internal: terminal actions at PacketContinue");

  Gen g{prog, "", ""};
  // gen_packet_filter (packet_filter.rs:7-29) + add_root_pred (utils.rs:363-379)
  bool any_pkt_child = false;
  for (auto& c : root.children) any_pkt_child = any_pkt_child || c.pred.on_packet();
  bool root_body = !root.actions.drop() || !root.deliver.empty();
  bool body_nonempty = root_body || any_pkt_child;
  prog.wraps_ethernet = body_nonempty && any_pkt_child;
  int d = prog.wraps_ethernet ? 2 : 1;
  if (prog.wraps_ethernet) {
    g.hip += "  if (v.eth_ok) {\n";
    g.rust += "  if let Ok(ethernet) = parse_to::<Ethernet>(mbuf) {\n";
  }
  if (root_body) g.update_body(root, d);
  g.children(root, d);
  if (prog.wraps_ethernet) {
    g.hip += "  }\n";
    g.rust += "  }\n";
  }
  prog.hip_body_branchy = "__device__ __forceinline__ void rtn_filter(const rtn_view& v, rtn_u32& act, rtn_u64* dm) {\n"
                          "  (void)v; (void)dm; RTN_KZ_DECL(v)\n" +
                          g.hip + "}\n";
  for (int form : {0, 1, 2}) {  // plain chain, range runs (the product), range runs + folded actions
    g.hip.clear();
    g.flat_pc_stmt = 0;
    g.act_flags.clear();
    g.range_runs = form >= 1;
    g.fold_act = form == 2;
    const std::string R0 = prog.wraps_ethernet ? "v.eth_ok" : "true";
    if (root_body) g.pc_flat_body(root, R0);
    g.pc_flat(root, R0);
    if (g.flat_pc_stmt != prog.delivers.size()) throw FilterError("internal: packet-continue statement count");
    (form == 0 ? prog.hip_body_chain : form == 1 ? prog.hip_body : prog.hip_body_fold) =
        "__device__ __forceinline__ void rtn_filter(const rtn_view& v, rtn_u32& act, rtn_u64* dm) {\n"
        "  (void)v; (void)dm; RTN_KZ_DECL(v)\n" +
        g.act_prologue() + g.hip + g.act_epilogue() + "}\n";
  }
  // The straight-line form evaluates every node for every frame; the nested form skips subtrees
  // no lane of a wave enters. Past kFlatMaxNodes the second wins (large disjoint subtrees).
  if (prog.tree.size > kFlatMaxNodes) prog.hip_body = prog.hip_body_branchy;
  prog.rust_listing = "let mut result = Actions::new();\n" + g.rust + "result\n";

  // packet_filter: the same emission (gen_packet_filter with FilterLayer::Packet), evaluated on a
  // forwarded frame's L4Context view. Such a frame always parses as Ethernet, so add_root_pred's
  // wrap is a no-op here.
  Gen gc{prog, "", "", FilterLayer::Packet};
  const PNode& croot = prog.conn_tree.root;
  bool c_any_pkt = false;
  for (auto& c : croot.children) c_any_pkt = c_any_pkt || c.pred.on_packet();
  if (!croot.actions.drop() || !croot.deliver.empty()) gc.update_body(croot, 1);  // packet_filter.rs:15-17
  gc.children(croot, 1);
  if (prog.conn_tree.size <= kFlatMaxNodes) {
    gc.hip.clear();
    if (!croot.actions.drop() || !croot.deliver.empty()) gc.conn_flat_body(croot, "true");
    gc.conn_flat(croot, "true");
    if (gc.flat_conn_stmt != prog.conn_delivers.size()) throw FilterError("internal: packet-filter statement count");
  }
  prog.hip_conn_body =
      "__device__ __forceinline__ void rtn_conn_filter(const rtn_cview& c, rtn_u32& data, rtn_u32& term, rtn_u64* cm) "
      "{\n  (void)c; (void)cm; RTN_KZ_DECL(c)\n" + gc.hip + "}\n";
  prog.rust_conn_listing = "let mut result = Actions::new();\n" +
                           std::string(c_any_pkt ? "if let Ok(ethernet) = parse_to::<Ethernet>(mbuf) {\n" : "") + gc.rust +
                           (c_any_pkt ? "}\n" : "") + "result\n";

  // packet_deliver (gen_deliver_filter, deliver_filter.rs:9-29): the root's deliveries, then its
  // children; add_root_pred's Ethernet wrap (utils.rs:363-379) always parses for a tracked frame
  Gen gd{prog, "", "", FilterLayer::PacketDeliver};
  const PNode& droot = prog.pd_tree.root;
  bool d_any_pkt = false;
  for (auto& c : droot.children) d_any_pkt = d_any_pkt || c.pred.on_packet();
  if (!droot.deliver.empty()) gd.pd_update_body(droot, 1, "1u", {});
  gd.pd_children(droot, 1, "1u", {});
  gd.hip.clear();
  gd.pd_flat_body(droot, "true", "1u");
  gd.pd_flat(droot, "true", "1u");
  if (gd.flat_stmt != prog.pd_stmts.size()) throw FilterError("internal: packet-deliver statement count");
  const bool d_wrap = !gd.rust.empty() && d_any_pkt;
  prog.hip_pd_body =
      "__device__ __forceinline__ void rtn_pd_filter(const rtn_cview& c, bool pok, const rtn_u32* f, rtn_u32* cnt) "
      "{\n  (void)c; (void)pok; (void)f; (void)cnt; RTN_KZ_DECL(c)\n" + gd.hip + "}\n";
  prog.rust_pd_listing = std::string(d_wrap ? "if let Ok(ethernet) = parse_to::<Ethernet>(mbuf) {\n" : "") + gd.rust +
                         (d_wrap ? "}\n" : "");
  return prog;
}

}  // namespace rtn
