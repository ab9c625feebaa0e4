// Filter AST for the packet-stage filter compiler.
//
// Restates the semantics of the reference filter language (stanford-esrg/retina):
//   core/src/filter/ast.rs:19-46      LAYERS protocol graph, has_path
//   core/src/filter/ast.rs:78-452     Predicate, on_packet/on_proto/on_session, is_excl, is_child
//   core/src/filter/ast.rs:455-832    is_excl_* / is_parent_* helpers
//   core/src/filter/ast.rs:834-950    Display / ProtocolName / FieldName / BinOp / Value
// Orderings replicate Rust's derived Ord (variant order, then fields in declaration order),
// because the reference sorts and dedups patterns with it (core/src/filter/mod.rs:127-128).
#pragma once

#include <array>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace rtn {

struct FilterError : std::runtime_error {
  explicit FilterError(const std::string& m) : std::runtime_error(m) {}
};

enum class BinOp : uint8_t { Eq, Ne, Ge, Le, Gt, Lt, In, Re, En, ByteRe, Contains, NotContains };
const char* binop_str(BinOp op);

struct Ipv4Net {
  uint32_t addr = 0;  // host-order value of the address as written (host bits kept, like ipnet)
  uint8_t prefix = 32;
  uint32_t netmask() const { return prefix == 0 ? 0u : (~0u << (32 - prefix)); }
  uint32_t network() const { return addr & netmask(); }
  uint32_t broadcast() const { return addr | ~netmask(); }
  bool contains(const Ipv4Net& o) const { return network() <= o.network() && o.broadcast() <= broadcast(); }
  bool operator==(const Ipv4Net& o) const { return addr == o.addr && prefix == o.prefix; }
};

struct U128 {
  uint64_t hi = 0, lo = 0;
  bool operator==(const U128& o) const { return hi == o.hi && lo == o.lo; }
  bool operator<(const U128& o) const { return hi != o.hi ? hi < o.hi : lo < o.lo; }
  bool operator<=(const U128& o) const { return !(o < *this); }
  U128 operator&(const U128& o) const { return {hi & o.hi, lo & o.lo}; }
  U128 operator|(const U128& o) const { return {hi | o.hi, lo | o.lo}; }
  U128 operator~() const { return {~hi, ~lo}; }
  std::string to_dec() const;
};

struct Ipv6Net {
  U128 addr;
  uint8_t prefix = 128;
  U128 netmask() const;
  U128 network() const { return addr & netmask(); }
  U128 broadcast() const { return addr | ~netmask(); }
  bool contains(const Ipv6Net& o) const { return network() <= o.network() && o.broadcast() <= broadcast(); }
  bool operator==(const Ipv6Net& o) const { return addr == o.addr && prefix == o.prefix; }
};

enum class VKind : uint8_t { Int, IntRange, Ipv4, Ipv6, Text, Byte };

struct Value {
  VKind kind = VKind::Int;
  uint64_t i = 0, to = 0;  // Int: i; IntRange: i..=to
  Ipv4Net v4;
  Ipv6Net v6;
  std::string text;
  std::vector<uint8_t> bytes;
  bool operator==(const Value& o) const;
  bool operator<(const Value& o) const;
  std::string str() const;
};

struct Predicate {
  bool binary = false;
  std::string protocol;
  std::string field;  // binary only
  BinOp op = BinOp::Eq;
  Value value;

  static Predicate unary(const std::string& proto) {
    Predicate p;
    p.protocol = proto;
    return p;
  }
  bool is_unary() const { return !binary; }
  bool is_binary() const { return binary; }
  bool operator==(const Predicate& o) const;
  bool operator!=(const Predicate& o) const { return !(*this == o); }
  bool operator<(const Predicate& o) const;
  std::string str() const;

  bool needs_conntrack() const;
  bool on_packet() const { return !needs_conntrack(); }
  bool on_proto() const { return needs_conntrack() && is_unary(); }
  bool on_session() const { return needs_conntrack() && is_binary(); }
  bool req_packet() const;
  bool is_excl(const Predicate& pred) const;
  bool is_child(const Predicate& pred) const;
};

// LAYERS graph (core/src/filter/ast.rs:19-46). Edges point from inner protocol to outer.
const std::vector<std::string>& layer_nodes();
int layer_index(const std::string& proto);  // -1 if unknown
bool layer_edge(int inner, int outer);
bool has_path(const std::string& from, const std::string& to);
// All simple paths from `from` to `to` (node index lists), like petgraph::algo::all_simple_paths.
std::vector<std::vector<int>> all_simple_paths(int from, int to);

// Rust std::net parsers (strict forms used by the reference's FromStr calls).
bool parse_rust_ipv4(const std::string& s, uint32_t& out);
bool parse_rust_ipv6(const std::string& s, U128& out);
std::string fmt_ipv4(uint32_t a);
std::string fmt_ipv6(const U128& a);

}  // namespace rtn
