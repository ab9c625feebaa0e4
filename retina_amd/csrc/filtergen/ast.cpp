// Filter AST semantics. See ast.hpp for the reference file:line map.
#include "ast.hpp"

#include <algorithm>
#include <cstdio>
#include <regex>
#include <string>

namespace rtn {

const char* binop_str(BinOp op) {
  switch (op) {
    case BinOp::Eq: return "=";
    case BinOp::Ne: return "!=";
    case BinOp::Ge: return ">=";
    case BinOp::Le: return "<=";
    case BinOp::Gt: return ">";
    case BinOp::Lt: return "<";
    case BinOp::In: return "in";
    case BinOp::Re: return "matches";
    case BinOp::En: return "eq";
    case BinOp::ByteRe: return "~b";
    case BinOp::Contains: return "contains";
    case BinOp::NotContains: return "not contains";
  }
  return "?";
}

std::string U128::to_dec() const {
  if (hi == 0) return std::to_string(lo);
  // repeated division by 10 on a 128-bit value
  uint64_t h = hi, l = lo;
  std::string s;
  while (h != 0 || l != 0) {
    unsigned __int128 v = ((unsigned __int128)h << 64) | l;
    unsigned rem = (unsigned)(v % 10);
    v /= 10;
    h = (uint64_t)(v >> 64);
    l = (uint64_t)v;
    s.push_back(char('0' + rem));
  }
  std::reverse(s.begin(), s.end());
  return s;
}

U128 Ipv6Net::netmask() const {
  if (prefix == 0) return {0, 0};
  if (prefix >= 128) return {~0ull, ~0ull};
  if (prefix <= 64) return {prefix == 64 ? ~0ull : (~0ull << (64 - prefix)), 0};
  return {~0ull, ~0ull << (128 - prefix)};
}

// ---------------------------------------------------------------------------------------------
// Value ordering / display (derive(Ord) on `enum Value`, ast.rs:920-950)

static int vkind_rank(VKind k) { return (int)k; }

bool Value::operator==(const Value& o) const {
  if (kind != o.kind) return false;
  switch (kind) {
    case VKind::Int: return i == o.i;
    case VKind::IntRange: return i == o.i && to == o.to;
    case VKind::Ipv4: return v4 == o.v4;
    case VKind::Ipv6: return v6 == o.v6;
    case VKind::Text: return text == o.text;
    case VKind::Byte: return bytes == o.bytes;
  }
  return false;
}

bool Value::operator<(const Value& o) const {
  if (kind != o.kind) return vkind_rank(kind) < vkind_rank(o.kind);
  switch (kind) {
    case VKind::Int: return i < o.i;
    case VKind::IntRange: return i != o.i ? i < o.i : to < o.to;
    case VKind::Ipv4: return v4.addr != o.v4.addr ? v4.addr < o.v4.addr : v4.prefix < o.v4.prefix;
    case VKind::Ipv6: return !(v6.addr == o.v6.addr) ? v6.addr < o.v6.addr : v6.prefix < o.v6.prefix;
    case VKind::Text: return text < o.text;
    case VKind::Byte: return bytes < o.bytes;
  }
  return false;
}

std::string fmt_ipv4(uint32_t a) {
  char b[32];
  snprintf(b, sizeof b, "%u.%u.%u.%u", a >> 24, (a >> 16) & 255, (a >> 8) & 255, a & 255);
  return b;
}

// Rust's Ipv6Addr Display (RFC 5952 style; ::ffff:a.b.c.d for IPv4-mapped).
std::string fmt_ipv6(const U128& a) {
  uint16_t seg[8];
  for (int k = 0; k < 4; ++k) seg[k] = (uint16_t)(a.hi >> (48 - 16 * k));
  for (int k = 0; k < 4; ++k) seg[4 + k] = (uint16_t)(a.lo >> (48 - 16 * k));
  bool all0 = true;
  for (int k = 0; k < 8; ++k) all0 = all0 && seg[k] == 0;
  if (all0) return "::";
  bool lb = true;
  for (int k = 0; k < 7; ++k) lb = lb && seg[k] == 0;
  if (lb && seg[7] == 1) return "::1";
  if (seg[0] == 0 && seg[1] == 0 && seg[2] == 0 && seg[3] == 0 && seg[4] == 0 && seg[5] == 0xffff) {
    return "::ffff:" + fmt_ipv4(((uint32_t)seg[6] << 16) | seg[7]);
  }
  int best_s = -1, best_l = 0, cur_s = -1, cur_l = 0;
  for (int k = 0; k < 8; ++k) {
    if (seg[k] == 0) {
      if (cur_l == 0) cur_s = k;
      ++cur_l;
      if (cur_l > best_l) { best_l = cur_l; best_s = cur_s; }
    } else {
      cur_l = 0;
    }
  }
  std::string s;
  char b[8];
  auto put = [&](int from, int to) {
    for (int k = from; k < to; ++k) {
      if (k != from) s += ":";
      snprintf(b, sizeof b, "%x", seg[k]);
      s += b;
    }
  };
  if (best_l > 1) {
    put(0, best_s);
    s += "::";
    put(best_s + best_l, 8);
  } else {
    put(0, 8);
  }
  return s;
}

std::string Value::str() const {
  switch (kind) {
    case VKind::Int: return std::to_string(i);
    case VKind::IntRange: return std::to_string(i) + ".." + std::to_string(to);
    case VKind::Ipv4: return fmt_ipv4(v4.addr) + "/" + std::to_string(v4.prefix);
    case VKind::Ipv6: return fmt_ipv6(v6.addr) + "/" + std::to_string(v6.prefix);
    case VKind::Text: return text;
    case VKind::Byte: {
      std::string s = "|";
      char b[4];
      for (size_t k = 0; k < bytes.size(); ++k) {
        if (k) s += " ";
        snprintf(b, sizeof b, "%02X", bytes[k]);
        s += b;
      }
      return s + "|";
    }
  }
  return "";
}

// ---------------------------------------------------------------------------------------------
// Predicate (derive(Ord) on `enum Predicate`, ast.rs:78-90)

bool Predicate::operator==(const Predicate& o) const {
  if (binary != o.binary || protocol != o.protocol) return false;
  if (!binary) return true;
  return field == o.field && op == o.op && value == o.value;
}

bool Predicate::operator<(const Predicate& o) const {
  if (binary != o.binary) return !binary;  // Unary < Binary
  if (protocol != o.protocol) return protocol < o.protocol;
  if (!binary) return false;
  if (field != o.field) return field < o.field;
  if (op != o.op) return (int)op < (int)o.op;
  return value < o.value;
}

std::string Predicate::str() const {
  if (!binary) return protocol;
  return protocol + "." + field + " " + binop_str(op) + " " + value.str();
}

// LAYERS (ast.rs:19-46): node insertion order matters for nothing but indices.
const std::vector<std::string>& layer_nodes() {
  static const std::vector<std::string> n = {"ethernet", "ipv4", "ipv6", "tcp", "udp",
                                             "tls",      "http", "dns",  "quic", "ssh"};
  return n;
}

int layer_index(const std::string& proto) {
  const auto& n = layer_nodes();
  for (size_t k = 0; k < n.size(); ++k)
    if (n[k] == proto) return (int)k;
  return -1;
}

static const std::vector<std::pair<int, int>>& layer_edges() {
  // (inner, outer)
  static const std::vector<std::pair<int, int>> e = {
      {1, 0}, {2, 0}, {3, 1}, {3, 2}, {4, 1}, {4, 2}, {5, 3}, {6, 3}, {7, 4}, {7, 3}, {8, 4}, {9, 3},
  };
  return e;
}

bool layer_edge(int inner, int outer) {
  for (auto& e : layer_edges())
    if (e.first == inner && e.second == outer) return true;
  return false;
}

static void dfs_paths(int cur, int to, std::vector<int>& path, std::vector<bool>& vis,
                      std::vector<std::vector<int>>& out) {
  for (auto& e : layer_edges()) {
    if (e.first != cur) continue;
    int nx = e.second;
    if (vis[nx]) continue;
    if (nx == to) {
      auto p = path;
      p.push_back(nx);
      out.push_back(p);
      continue;
    }
    vis[nx] = true;
    path.push_back(nx);
    dfs_paths(nx, to, path, vis, out);
    path.pop_back();
    vis[nx] = false;
  }
}

std::vector<std::vector<int>> all_simple_paths(int from, int to) {
  std::vector<std::vector<int>> out;
  std::vector<int> path{from};
  std::vector<bool> vis(layer_nodes().size(), false);
  vis[from] = true;
  dfs_paths(from, to, path, vis, out);
  return out;
}

bool has_path(const std::string& from, const std::string& to) {
  int f = layer_index(from), t = layer_index(to);
  if (f < 0 || t < 0) return false;
  return !all_simple_paths(f, t).empty();
}

bool Predicate::needs_conntrack() const { return has_path(protocol, "tcp") || has_path(protocol, "udp"); }

// ast.rs:120-136 with ConnData::supported_fields/protocols (protocols/stream/mod.rs:154-167)
bool Predicate::req_packet() const {
  if (!on_packet()) return false;
  if (binary) {
    static const char* conn_fields[] = {"src_port", "dst_port", "src_addr", "dst_addr"};
    for (auto f : conn_fields)
      if (field == f) return false;
    return field != "port" && field != "addr";
  }
  static const char* conn_protos[] = {"ipv4", "ipv6", "tcp", "udp"};
  for (auto p : conn_protos)
    if (protocol == p) return false;
  return true;
}

// --------------------------------------------------------------------------------------------- is_excl

static bool is_excl_int(uint64_t from, uint64_t to, BinOp op, uint64_t pf, uint64_t pt, BinOp pop) {
  switch (op) {
    case BinOp::Eq:
      switch (pop) {
        case BinOp::Eq: return from != pf;
        case BinOp::Ne: return from == pf;
        case BinOp::In: return from < pf || from > pt;
        case BinOp::Ge: return pf > from;
        case BinOp::Le: return pf < from;
        case BinOp::Gt: return pf >= from;
        case BinOp::Lt: return pf <= from;
        default: break;
      }
      break;
    case BinOp::Ne:
      if (pop == BinOp::Eq) return from == pf;
      break;
    case BinOp::Ge:
      switch (pop) {
        case BinOp::Le: case BinOp::In: case BinOp::Eq: return from > pt;
        case BinOp::Lt: return from >= pf;
        default: break;
      }
      break;
    case BinOp::Le:
      switch (pop) {
        case BinOp::Ge: case BinOp::In: case BinOp::Eq: return from < pf;
        case BinOp::Gt: return from <= pf;
        default: break;
      }
      break;
    case BinOp::Gt:
      switch (pop) {
        case BinOp::Le: case BinOp::In: case BinOp::Eq: return from >= pt;
        case BinOp::Lt: return from > pf;
        default: break;
      }
      break;
    case BinOp::Lt:
      switch (pop) {
        case BinOp::Ge: case BinOp::In: case BinOp::Eq: return from <= pf;
        case BinOp::Gt: return from <= pf + 1;  // u64 wrap like release-mode Rust
        default: break;
      }
      break;
    case BinOp::In:
      switch (pop) {
        case BinOp::Eq: return pf < from || pf > to;
        case BinOp::Ge: return pf > to;
        case BinOp::Gt: return pf >= to;
        case BinOp::Le: return pf < from;
        case BinOp::Lt: return pf <= from;
        case BinOp::In: return pt < from || pf > to;
        default: break;
      }
      break;
    default: break;
  }
  return false;
}

template <class Net>
static bool is_excl_ip(const Net& a, BinOp op, const Net& b, BinOp pop) {
  bool eqin = op == BinOp::Eq || op == BinOp::In;
  bool peqin = pop == BinOp::Eq || pop == BinOp::In;
  if (eqin) {
    if (peqin) return !b.contains(a) && !a.contains(b);
    if (pop == BinOp::Ne) return b == a;
    return false;
  }
  if (op == BinOp::Ne && peqin) return b == a;
  return false;
}

static bool regex_match(const std::string& re, const std::string& txt) {
  // Approximation of the Rust `regex` crate with ECMAScript std::regex (search semantics).
  try {
    return std::regex_search(txt, std::regex(re));
  } catch (const std::regex_error&) {
    throw FilterError("Invalid Regex string " + re);
  }
}

static bool is_excl_text(const std::string& t, BinOp op, const std::string& pt, BinOp pop) {
  if (op == BinOp::Eq && pop == BinOp::Eq) return pt != t;
  if ((op == BinOp::Ne && pop == BinOp::Eq) || (op == BinOp::Eq && pop == BinOp::Ne)) return pt == t;
  if (op == BinOp::Ne || pop == BinOp::Ne) return false;
  if (op == BinOp::Re && pop == BinOp::Re) return false;
  if (op == BinOp::Contains && pop == BinOp::Eq) return pt.find(t) == std::string::npos;
  if (op == BinOp::Eq && pop == BinOp::Contains) return t.find(pt) == std::string::npos;
  if (op == BinOp::Contains && pop == BinOp::Contains) return false;
  if ((op == BinOp::Re && pop == BinOp::Contains) || (op == BinOp::Contains && pop == BinOp::Re)) return false;
  const std::string& re = op == BinOp::Re ? t : pt;
  const std::string& txt = op == BinOp::Re ? pt : t;
  return !regex_match(re, txt);
}

static bool bytes_find(const std::vector<uint8_t>& needle, const std::vector<uint8_t>& hay) {
  if (needle.empty()) return true;
  return std::search(hay.begin(), hay.end(), needle.begin(), needle.end()) != hay.end();
}

static bool is_excl_byte(const std::vector<uint8_t>& b, BinOp op, const std::vector<uint8_t>& pb, BinOp pop) {
  if (op == BinOp::Eq && pop == BinOp::Eq) return pb != b;
  if ((op == BinOp::Ne && pop == BinOp::Eq) || (op == BinOp::Eq && pop == BinOp::Ne)) return pb == b;
  if (op == BinOp::Ne || pop == BinOp::Ne) return false;
  if (op == BinOp::Contains && pop == BinOp::Eq) return !bytes_find(b, pb);
  if (op == BinOp::Eq && pop == BinOp::Contains) return !bytes_find(pb, b);
  return false;
}

// ast.rs:215-309
bool Predicate::is_excl(const Predicate& pred) const {
  if (is_unary() && pred.is_unary()) return true;
  if (is_unary() != pred.is_unary()) return false;
  if (protocol != pred.protocol) return false;
  if (field != pred.field) return false;
  const Value& v = value;
  const Value& pv = pred.value;
  switch (v.kind) {
    case VKind::Int:
      if (pv.kind == VKind::Int) return is_excl_int(v.i, v.i, op, pv.i, pv.i, pred.op);
      if (pv.kind == VKind::IntRange) return is_excl_int(v.i, v.i, op, pv.i, pv.to, pred.op);
      return false;
    case VKind::IntRange:
      if (pv.kind == VKind::Int) return is_excl_int(v.i, v.to, op, pv.i, pv.i, pred.op);
      if (pv.kind == VKind::IntRange) return is_excl_int(v.i, v.to, op, pv.i, pv.to, pred.op);
      return false;
    case VKind::Ipv4:
      return pv.kind == VKind::Ipv4 && is_excl_ip(v.v4, op, pv.v4, pred.op);
    case VKind::Ipv6:
      return pv.kind == VKind::Ipv6 && is_excl_ip(v.v6, op, pv.v6, pred.op);
    case VKind::Text:
      return pv.kind == VKind::Text && is_excl_text(v.text, op, pv.text, pred.op);
    case VKind::Byte:
      return pv.kind == VKind::Byte && is_excl_byte(v.bytes, op, pv.bytes, pred.op);
  }
  return false;
}

// --------------------------------------------------------------------------------------------- is_child

static bool is_parent_int(uint64_t cf, uint64_t ct, BinOp cop, uint64_t pf, uint64_t pt, BinOp pop) {
  switch (cop) {
    case BinOp::Eq:
    case BinOp::In:
      if (pop == BinOp::Ge) return pf <= cf;
      if (pop == BinOp::Gt) return pf < cf;
      if (pop == BinOp::Le) return pf >= ct;
      if (pop == BinOp::Lt) return pf > ct;
      if (pop == BinOp::In) return pf <= cf && pt >= ct;
      break;
    case BinOp::Ge:
      if (pop == BinOp::Ge || pop == BinOp::Gt) return pf < cf;
      break;
    case BinOp::Le:
      if (pop == BinOp::Le || pop == BinOp::Lt) return pf > cf;
      break;
    case BinOp::Gt:
      if (pop == BinOp::Gt || pop == BinOp::Ge) return pf <= cf;
      break;
    case BinOp::Lt:
      if (pop == BinOp::Le || pop == BinOp::Lt) return pf >= cf;
      break;
    default: break;
  }
  return false;
}

template <class Net>
static bool is_parent_ip(const Net& c, BinOp cop, const Net& p, BinOp pop) {
  if (cop == BinOp::Eq || cop == BinOp::In) {
    if (pop == BinOp::Eq || pop == BinOp::In) return p.contains(c);
  } else if (cop == BinOp::Ne) {
    if (pop == BinOp::Ne) return p.contains(c);
  }
  return false;
}

static bool is_parent_text(const std::string& ct, BinOp cop, const std::string& pt, BinOp pop) {
  if (pop == BinOp::Contains && (cop == BinOp::Eq || cop == BinOp::Contains)) return ct.find(pt) != std::string::npos;
  if (pop != BinOp::Re || cop != BinOp::Eq) return false;
  return regex_match(pt, ct);
}

static bool is_parent_bytes(const std::vector<uint8_t>& cb, BinOp cop, const std::vector<uint8_t>& pb, BinOp pop) {
  if (pop == BinOp::Contains && (cop == BinOp::Eq || cop == BinOp::Contains)) return bytes_find(pb, cb);
  return false;
}

// ast.rs:312-452
bool Predicate::is_child(const Predicate& pred) const {
  if (protocol != pred.protocol) return false;
  if (*this == pred) return false;
  if (is_binary() && pred.is_binary()) {
    if (field != pred.field) return false;
    BinOp pop = pred.op;
    if (pop == BinOp::Ne) return false;
    if (pop == BinOp::Eq && pred.value.kind != VKind::Ipv4 && pred.value.kind != VKind::Ipv6) return false;
    if (op == BinOp::Ne || pop == BinOp::Ne) return false;
    if (op == BinOp::En || pop == BinOp::En) return false;
    if (op == BinOp::Re && pop == BinOp::Re) return false;
    if ((op == BinOp::Ge || op == BinOp::Gt) && (pop == BinOp::Le || pop == BinOp::Lt)) return false;
    if ((pop == BinOp::Ge || pop == BinOp::Gt) && (op == BinOp::Le || op == BinOp::Lt)) return false;
    const Value& v = value;
    const Value& pv = pred.value;
    switch (v.kind) {
      case VKind::Int:
        if (pv.kind == VKind::Int) return is_parent_int(v.i, v.i, op, pv.i, pv.i, pop);
        if (pv.kind == VKind::IntRange) return is_parent_int(v.i, v.i, op, pv.i, pv.to, pop);
        return false;
      case VKind::IntRange:
        if (pv.kind == VKind::Int) return is_parent_int(v.i, v.to, op, pv.i, pv.i, pop);
        if (pv.kind == VKind::IntRange) return is_parent_int(v.i, v.to, op, pv.i, pv.to, pop);
        return false;
      case VKind::Ipv4: return pv.kind == VKind::Ipv4 && is_parent_ip(v.v4, op, pv.v4, pop);
      case VKind::Ipv6: return pv.kind == VKind::Ipv6 && is_parent_ip(v.v6, op, pv.v6, pop);
      case VKind::Text: return pv.kind == VKind::Text && is_parent_text(v.text, op, pv.text, pop);
      case VKind::Byte: return pv.kind == VKind::Byte && is_parent_bytes(v.bytes, op, pv.bytes, pop);
    }
  }
  return is_binary() && pred.is_unary();
}

// --------------------------------------------------------------------------------------------- Rust std::net parsers

namespace {
struct NetParser {
  const std::string& s;
  size_t pos = 0;
  explicit NetParser(const std::string& str) : s(str) {}
  bool peek(char c) const { return pos < s.size() && s[pos] == c; }
  static int digit(char c, int radix) {
    int d = -1;
    if (c >= '0' && c <= '9') d = c - '0';
    else if (c >= 'a' && c <= 'z') d = c - 'a' + 10;
    else if (c >= 'A' && c <= 'Z') d = c - 'A' + 10;
    return (d >= 0 && d < radix) ? d : -1;
  }
  // core::net::parser::read_number (atomic)
  bool read_number(int radix, int max_digits, bool allow_zero_prefix, uint32_t max_val, uint32_t& out) {
    size_t save = pos;
    int count = 0;
    bool lead0 = peek('0');
    uint64_t v = 0;
    while (pos < s.size() && count < max_digits) {
      int d = digit(s[pos], radix);
      if (d < 0) break;
      v = v * radix + d;
      if (v > max_val) { pos = save; return false; }
      ++pos;
      ++count;
    }
    if (count == 0 || (!allow_zero_prefix && lead0 && count > 1)) { pos = save; return false; }
    out = (uint32_t)v;
    return true;
  }
  bool read_ipv4(uint32_t& out) {
    size_t save = pos;
    uint32_t a = 0;
    for (int k = 0; k < 4; ++k) {
      if (k > 0) {
        if (!peek('.')) { pos = save; return false; }
        ++pos;
      }
      uint32_t o;
      if (!read_number(10, 3, false, 255, o)) { pos = save; return false; }
      a = (a << 8) | o;
    }
    out = a;
    return true;
  }
  // returns (count, ipv4_embedded)
  std::pair<int, bool> read_groups(uint16_t* groups, int limit) {
    for (int i = 0; i < limit; ++i) {
      if (i < limit - 1) {
        size_t save = pos;
        bool ok = true;
        if (i > 0) {
          if (peek(':')) ++pos; else ok = false;
        }
        uint32_t v4;
        if (ok && read_ipv4(v4)) {
          groups[i] = (uint16_t)(v4 >> 16);
          groups[i + 1] = (uint16_t)v4;
          return {i + 2, true};
        }
        pos = save;
      }
      size_t save = pos;
      bool ok = true;
      if (i > 0) {
        if (peek(':')) ++pos; else ok = false;
      }
      uint32_t g;
      if (!ok || !read_number(16, 4, true, 0xffff, g)) { pos = save; return {i, false}; }
      groups[i] = (uint16_t)g;
    }
    return {limit, false};
  }
  bool read_ipv6(U128& out) {
    uint16_t head[8] = {0};
    auto [hs, h4] = read_groups(head, 8);
    if (hs < 8) {
      if (h4) return false;
      if (!peek(':')) return false;
      ++pos;
      if (!peek(':')) return false;
      ++pos;
      uint16_t tail[7] = {0};
      int limit = 8 - (hs + 1);
      auto [ts, t4] = read_groups(tail, limit);
      (void)t4;
      for (int k = 0; k < ts; ++k) head[8 - ts + k] = tail[k];
    }
    out.hi = ((uint64_t)head[0] << 48) | ((uint64_t)head[1] << 32) | ((uint64_t)head[2] << 16) | head[3];
    out.lo = ((uint64_t)head[4] << 48) | ((uint64_t)head[5] << 32) | ((uint64_t)head[6] << 16) | head[7];
    return true;
  }
};
}  // namespace

bool parse_rust_ipv4(const std::string& s, uint32_t& out) {
  NetParser p(s);
  return p.read_ipv4(out) && p.pos == s.size();
}

bool parse_rust_ipv6(const std::string& s, U128& out) {
  NetParser p(s);
  return p.read_ipv6(out) && p.pos == s.size();
}

}  // namespace rtn
