// Filter-string parser: a hand-written PEG that accepts exactly the language of the reference
// grammar (core/src/filter/grammar.pest:5-75, pest 2.5 semantics: ordered choice, greedy
// non-backtracking repetition, implicit WHITESPACE = " " | NEWLINE between tokens of
// non-atomic rules) and builds the same disjunctive normal form as
// core/src/filter/parser.rs:94-357 (FilterParser::parse_filter / flatten_*).
#include <memory>

#include "filter.hpp"

namespace rtn {
namespace {

struct Node {
  enum Kind { Pred, Disj, Conj } kind;
  Predicate pred;
  std::vector<Node> kids;
};

class Peg {
 public:
  explicit Peg(const std::string& s) : s_(s) {}

  // filter = _{ SOI ~ expr? ~ EOI }   -> returns Disjunct (possibly empty)
  Node parse_filter() {
    size_t p = 0;
    p = ws(p);
    Node root{Node::Disj, {}, {}};
    size_t q;
    Node e;
    if (expr(p, q, e)) {
      p = ws(q);
      root = e;
    }
    if (p != s_.size()) throw FilterError("Invalid filter format");
    return root;
  }

 private:
  const std::string& s_;

  bool at(size_t p, const char* lit) const { return s_.compare(p, strlen_(lit), lit) == 0; }
  static size_t strlen_(const char* l) {
    size_t n = 0;
    while (l[n]) ++n;
    return n;
  }
  // WHITESPACE = _{ " " | NEWLINE }, NEWLINE = "\n" | "\r\n" | "\r"
  size_t ws(size_t p) const {
    while (p < s_.size()) {
      if (s_[p] == ' ' || s_[p] == '\n' || s_[p] == '\r') ++p;
      else break;
    }
    return p;
  }
  static bool alpha(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }
  static bool digit(char c) { return c >= '0' && c <= '9'; }
  static bool alnum(char c) { return alpha(c) || digit(c); }
  static bool hexd(char c) { return digit(c) || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }

  // expr = { sub_expr ~ (or_op ~ sub_expr)* }
  bool expr(size_t p, size_t& out, Node& n) {
    Node d{Node::Disj, {}, {}};
    Node c;
    size_t q;
    if (!sub_expr(p, q, c)) return false;
    d.kids.push_back(c);
    p = q;
    for (;;) {
      size_t r = ws(p);
      size_t r2;
      if (!or_op(r, r2)) break;
      r2 = ws(r2);
      Node c2;
      size_t r3;
      if (!sub_expr(r2, r3, c2)) break;
      d.kids.push_back(c2);
      p = r3;
    }
    out = p;
    n = d;
    return true;
  }
  bool or_op(size_t p, size_t& out) {
    for (const char* l : {"||", "or", "OR"})
      if (at(p, l)) { out = p + strlen_(l); return true; }
    return false;
  }
  bool and_op(size_t p, size_t& out) {
    for (const char* l : {"&&", "and", "AND"})
      if (at(p, l)) { out = p + strlen_(l); return true; }
    return false;
  }
  // sub_expr = { term ~ (and_op ~ term)* } ; term = _{ predicate | "(" ~ expr ~ ")" }
  bool sub_expr(size_t p, size_t& out, Node& n) {
    Node c{Node::Conj, {}, {}};
    size_t q;
    if (!term(p, q, c)) return false;
    p = q;
    for (;;) {
      size_t r = ws(p);
      size_t r2;
      if (!and_op(r, r2)) break;
      r2 = ws(r2);
      size_t r3;
      Node tmp = c;
      if (!term(r2, r3, tmp)) break;
      c = tmp;
      p = r3;
    }
    out = p;
    n = c;
    return true;
  }
  // Appends the term's nodes to the conjunct (parser.rs:165-177, 179-238).
  bool term(size_t p, size_t& out, Node& conj) {
    size_t q;
    std::vector<Node> pn;
    if (predicate(p, q, pn)) {
      for (auto& x : pn) conj.kids.push_back(x);
      out = q;
      return true;
    }
    if (p < s_.size() && s_[p] == '(') {
      size_t r = ws(p + 1);
      Node e;
      size_t r2;
      if (!expr(r, r2, e)) return false;
      r2 = ws(r2);
      if (r2 < s_.size() && s_[r2] == ')') {
        conj.kids.push_back(e);
        out = r2 + 1;
        return true;
      }
    }
    return false;
  }
  // identifier = @{ ASCII_ALPHA ~ (ASCII_ALPHANUMERIC | "_")* }
  bool ident(size_t p, size_t& out) const {
    if (p >= s_.size() || !alpha(s_[p])) return false;
    ++p;
    while (p < s_.size() && (alnum(s_[p]) || s_[p] == '_')) ++p;
    out = p;
    return true;
  }
  // predicate = { protocol ~ ("." ~ (combined_field | field) ~ bin_op ~ value)? }
  bool predicate(size_t p, size_t& out, std::vector<Node>& nodes) {
    size_t q;
    if (!ident(p, q)) return false;
    std::string proto = s_.substr(p, q - p);
    // optional group
    size_t g = ws(q);
    bool have = false;
    std::string field;
    bool combined = false;
    BinOp op = BinOp::Eq;
    Value val;
    size_t gend = q;
    if (g < s_.size() && s_[g] == '.') {
      size_t f0 = ws(g + 1), f1 = 0;
      bool fok = false;
      if (at(f0, "addr") || at(f0, "port")) {
        combined = true;
        f1 = f0 + 4;
        fok = true;
      } else if (ident(f0, f1)) {
        fok = true;
      }
      if (fok) {
        field = s_.substr(f0, f1 - f0);
        size_t o0 = ws(f1), o1;
        if (bin_op(o0, o1, op)) {
          size_t v0 = ws(o1), v1;
          if (value(v0, v1, val)) {
            have = true;
            gend = v1;
          }
        }
      }
    }
    if (!have) {
      nodes.push_back(Node{Node::Pred, Predicate::unary(proto), {}});
      out = q;
      return true;
    }
    out = gend;
    if (!combined) {
      Predicate pr;
      pr.binary = true;
      pr.protocol = proto;
      pr.field = field;
      pr.op = op;
      pr.value = val;
      nodes.push_back(Node{Node::Pred, pr, {}});
      return true;
    }
    Predicate src, dst;
    src.binary = dst.binary = true;
    src.protocol = dst.protocol = proto;
    src.field = "src_" + field;
    dst.field = "dst_" + field;
    src.op = dst.op = op;
    src.value = dst.value = val;
    if (op == BinOp::Ne) {
      nodes.push_back(Node{Node::Pred, src, {}});
      nodes.push_back(Node{Node::Pred, dst, {}});
    } else {
      Node c1{Node::Conj, {}, {Node{Node::Pred, src, {}}}};
      Node c2{Node::Conj, {}, {Node{Node::Pred, dst, {}}}};
      nodes.push_back(Node{Node::Disj, {}, {c1, c2}});
    }
    return true;
  }
  // bin_op order matters (grammar.pest:55-70)
  bool bin_op(size_t p, size_t& out, BinOp& op) {
    struct L { const char* s; BinOp op; };
    static const L lits[] = {
        {"=", BinOp::Eq},         {"!=", BinOp::Ne},         {"ne", BinOp::Ne},       {">=", BinOp::Ge},
        {"ge", BinOp::Ge},        {"<=", BinOp::Le},         {"le", BinOp::Le},       {">", BinOp::Gt},
        {"gt", BinOp::Gt},        {"<", BinOp::Lt},          {"lt", BinOp::Lt},       {"in", BinOp::In},
        {"~b", BinOp::ByteRe},    {"~", BinOp::Re},          {"matches", BinOp::Re},  {"eq", BinOp::En},
        {"contains", BinOp::Contains}, {"!contains", BinOp::NotContains}, {"not contains", BinOp::NotContains},
    };
    for (auto& l : lits)
      if (at(p, l.s)) {
        out = p + strlen_(l.s);
        op = l.op;
        return true;
      }
    return false;
  }
  // ipv4_addr = @{ ASCII_DIGIT{1,3} ~ ("." ~ ASCII_DIGIT{1,3}){3} }
  bool ipv4_addr(size_t p, size_t& out) const {
    for (int k = 0; k < 4; ++k) {
      if (k > 0) {
        if (p >= s_.size() || s_[p] != '.') return false;
        ++p;
      }
      int n = 0;
      while (n < 3 && p < s_.size() && digit(s_[p])) { ++p; ++n; }
      if (n == 0) return false;
    }
    out = p;
    return true;
  }
  // ipv6_addr = @{ (":" | ASCII_ALPHANUMERIC{1,4}) ~ ":" ~ (ipv4_addr | ASCII_ALPHANUMERIC{1,4} | ":")* }
  bool ipv6_addr(size_t p, size_t& out) const {
    if (p < s_.size() && s_[p] == ':') {
      ++p;
    } else {
      int n = 0;
      while (n < 4 && p < s_.size() && alnum(s_[p])) { ++p; ++n; }
      if (n == 0) return false;
    }
    if (p >= s_.size() || s_[p] != ':') return false;
    ++p;
    for (;;) {
      size_t q;
      if (ipv4_addr(p, q)) { p = q; continue; }
      int n = 0;
      size_t r = p;
      while (n < 4 && r < s_.size() && alnum(s_[r])) { ++r; ++n; }
      if (n > 0) { p = r; continue; }
      if (p < s_.size() && s_[p] == ':') { ++p; continue; }
      break;
    }
    out = p;
    return true;
  }
  bool digits(size_t p, size_t& out, int minn, int maxn) const {
    int n = 0;
    while ((maxn < 0 || n < maxn) && p < s_.size() && digit(s_[p])) { ++p; ++n; }
    if (n < minn) return false;
    out = p;
    return true;
  }
  static uint64_t parse_u64(const std::string& t) {
    uint64_t v = 0;
    for (char c : t) {
      uint64_t d = (uint64_t)(c - '0');
      if (v > (UINT64_MAX - d) / 10) throw FilterError("Invalid Integer");
      v = v * 10 + d;
    }
    return v;
  }
  static uint8_t parse_u8(const std::string& t) {
    uint64_t v = parse_u64(t);
    if (v > 255) throw FilterError("Invalid Integer");
    return (uint8_t)v;
  }
  // value = { ipv4_lit | ipv6_lit | int_range | int_lit | byte_lit | str_lit }
  bool value(size_t p, size_t& out, Value& v) {
    size_t q;
    if (ipv4_addr(p, q)) {
      std::string a = s_.substr(p, q - p);
      uint8_t prefix = 32;
      size_t e = q;
      if (q < s_.size() && s_[q] == '/') {
        size_t r;
        if (digits(q + 1, r, 1, 2)) {
          prefix = parse_u8(s_.substr(q + 1, r - q - 1));
          e = r;
        }
      }
      uint32_t ip;
      if (!parse_rust_ipv4(a, ip)) throw FilterError("Invalid Address");
      if (prefix > 32) throw FilterError("Invalid Prefix Len");
      v = Value();
      v.kind = VKind::Ipv4;
      v.v4.addr = ip;
      v.v4.prefix = prefix;
      out = e;
      return true;
    }
    if (ipv6_addr(p, q)) {
      std::string a = s_.substr(p, q - p);
      uint8_t prefix = 128;
      size_t e = q;
      if (q < s_.size() && s_[q] == '/') {
        size_t r;
        if (digits(q + 1, r, 1, 3)) {
          prefix = parse_u8(s_.substr(q + 1, r - q - 1));
          e = r;
        }
      }
      U128 ip;
      if (!parse_rust_ipv6(a, ip)) throw FilterError("Invalid Address");
      if (prefix > 128) throw FilterError("Invalid Prefix Len");
      v = Value();
      v.kind = VKind::Ipv6;
      v.v6.addr = ip;
      v.v6.prefix = prefix;
      out = e;
      return true;
    }
    size_t a1;
    if (digits(p, a1, 1, -1)) {
      // int_range = ${ int_lit ~ ".." ~ int_lit }
      size_t b1;
      if (at(a1, "..") && digits(a1 + 2, b1, 1, -1)) {
        uint64_t from = parse_u64(s_.substr(p, a1 - p));
        uint64_t to = parse_u64(s_.substr(a1 + 2, b1 - a1 - 2));
        if (from >= to)
          throw FilterError("Invalid Range: " + std::to_string(from) + ".." + std::to_string(to));
        v = Value();
        v.kind = VKind::IntRange;
        v.i = from;
        v.to = to;
        out = b1;
        return true;
      }
      v = Value();
      v.kind = VKind::Int;
      v.i = parse_u64(s_.substr(p, a1 - p));
      out = a1;
      return true;
    }
    // byte_lit = { "|" ~ (byte)+ ~ "|" } ; byte = { !("|") ~ ASCII_HEX_DIGIT{2} ~ " "? }
    if (p < s_.size() && s_[p] == '|') {
      // Non-atomic rules: implicit skips before each byte, between the lookahead and the first
      // hex digit, between the two hex digits (ASCII_HEX_DIGIT{2} expands to a sequence) and
      // before the optional " ".
      size_t r = p + 1;
      int nbytes = 0;
      for (;;) {
        size_t t = ws(r);
        if (t < s_.size() && s_[t] == '|') break;
        if (t >= s_.size() || !hexd(s_[t])) break;
        size_t t3 = ws(t + 1);
        if (t3 >= s_.size() || !hexd(s_[t3])) break;
        size_t t4 = ws(t3 + 1);
        if (t4 < s_.size() && s_[t4] == ' ') ++t4;
        r = t4;
        ++nbytes;
      }
      if (nbytes > 0) {
        size_t t = ws(r);
        if (t < s_.size() && s_[t] == '|') {
          std::string raw = s_.substr(p, t + 1 - p);
          std::vector<uint8_t> bytes;
          std::string tok;
          // parser.rs:295-307: strip '|', split_whitespace, u8::from_str_radix(tok, 16)
          auto flush = [&]() {
            if (tok.empty()) return;
            unsigned long v = 0;
            for (char ch : tok) {
              int d = (ch >= '0' && ch <= '9') ? ch - '0' : (ch >= 'a' && ch <= 'f') ? ch - 'a' + 10 : ch - 'A' + 10;
              v = v * 16 + (unsigned long)d;
              if (v > 255) throw FilterError("Failed to parse " + tok + " in " + raw);
            }
            bytes.push_back((uint8_t)v);
            tok.clear();
          };
          for (char c : raw) {
            if (c == '|') continue;
            if (c == ' ' || c == '\n' || c == '\r' || c == '\t') flush();
            else tok.push_back(c);
          }
          flush();
          v = Value();
          v.kind = VKind::Byte;
          v.bytes = bytes;
          out = t + 1;
          return true;
        }
      }
    }
    // str_lit = _{ "'" ~ text ~ "'" } ; text = { (!("'") ~ ANY)+ }
    if (p < s_.size() && s_[p] == '\'') {
      size_t t0 = ws(p + 1);
      size_t cur = t0;
      int iters = 0;
      for (;;) {
        size_t save = cur;
        size_t a = iters > 0 ? ws(cur) : cur;
        if (a < s_.size() && s_[a] == '\'') { cur = save; break; }
        a = ws(a);
        if (a >= s_.size()) { cur = save; break; }
        // ANY: one UTF-8 code point
        unsigned char c = (unsigned char)s_[a];
        size_t len = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : 4;
        cur = a + len;
        ++iters;
      }
      if (iters > 0) {
        size_t e = ws(cur);
        if (e < s_.size() && s_[e] == '\'') {
          v = Value();
          v.kind = VKind::Text;
          v.text = s_.substr(t0, cur - t0);
          out = e + 1;
          return true;
        }
      }
    }
    return false;
  }
};

void flatten_disjunct(const Node& d, std::vector<RawPattern>& out);

std::vector<RawPattern> flatten_conjunct(const Node& c) {
  std::vector<RawPattern> flat(1);
  for (const Node& t : c.kids) {
    if (t.kind == Node::Pred) {
      for (auto& fc : flat) fc.push_back(t.pred);
    } else if (t.kind == Node::Disj) {
      std::vector<RawPattern> fd;
      flatten_disjunct(t, fd);
      auto cur = flat;
      flat.clear();
      for (auto& conj : fd)
        for (auto& fc : cur) {
          RawPattern r = fc;
          r.insert(r.end(), conj.begin(), conj.end());
          flat.push_back(r);
        }
    } else {
      throw FilterError("Conjunct contains non-predicate or disjunct");
    }
  }
  return flat;
}

void flatten_disjunct(const Node& d, std::vector<RawPattern>& out) {
  for (const Node& c : d.kids) {
    auto f = flatten_conjunct(c);
    out.insert(out.end(), f.begin(), f.end());
  }
}

}  // namespace

std::vector<RawPattern> parse_filter_raw(const std::string& filter) {
  Peg peg(filter);
  Node root = peg.parse_filter();
  std::vector<RawPattern> out;
  flatten_disjunct(root, out);
  return out;
}

}  // namespace rtn
