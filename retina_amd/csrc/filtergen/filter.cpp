// Patterns, Filter::new, datatypes and subscription specs. See filter.hpp for the reference map.
#include "filter.hpp"

#include <algorithm>
#include <cstdio>
#include <sstream>

namespace rtn {

std::string FlatPattern::str() const {
  std::string s = "[";
  for (size_t k = 0; k < predicates.size(); ++k) {
    if (k) s += ", ";
    s += predicates[k].str();
  }
  return s + "]";
}

// pattern.rs:176-206
bool LayeredPattern::add_protocol(const std::string& proto, const std::vector<Predicate>& preds) {
  int node = layer_index(proto);
  if (node < 0) return false;
  bool ret = true;
  if (!layers.empty()) {
    int prev = layer_index(layers.back().first);
    if (prev < 0) return false;
    ret = ret && layer_edge(node, prev);
    for (auto& p : preds) ret = ret && p.is_binary() && p.protocol == proto;
  } else {
    ret = ret && layer_edge(node, layer_index("ethernet"));
  }
  if (!ret) return false;
  for (auto& l : layers)
    if (l.first == proto) {  // LinkedHashMap::insert on an existing key keeps its position
      l.second = preds;
      return true;
    }
  layers.emplace_back(proto, preds);
  return true;
}

FlatPattern LayeredPattern::to_flat() const {
  FlatPattern f;
  for (auto& l : layers) {
    f.predicates.push_back(Predicate::unary(l.first));
    f.predicates.insert(f.predicates.end(), l.second.begin(), l.second.end());
  }
  return f;
}

// pattern.rs:64-130
std::vector<LayeredPattern> to_fully_qualified(const FlatPattern& p) {
  std::vector<LayeredPattern> out;
  if (p.predicates.empty()) return out;
  std::set<std::string> headers;
  for (auto& pr : p.predicates) headers.insert(pr.protocol);
  const int eth = layer_index("ethernet");
  std::set<std::vector<int>> node_paths;
  for (auto& h : headers) {
    int node = layer_index(h);
    if (node < 0) throw FilterError("Predicate header invalid: " + h);
    for (auto& path : all_simple_paths(node, eth)) node_paths.insert(path);
  }
  std::set<std::vector<std::string>> fq_paths;
  for (auto& np : node_paths) {
    std::vector<std::string> fq;
    for (int n : np) fq.push_back(layer_nodes()[n]);
    fq.pop_back();  // remove ethernet
    std::reverse(fq.begin(), fq.end());
    fq_paths.insert(fq);
  }
  for (auto& fq : fq_paths) {
    std::set<std::string> fqh(fq.begin(), fq.end());
    bool subset = std::includes(fqh.begin(), fqh.end(), headers.begin(), headers.end());
    if (!subset) continue;
    LayeredPattern lp;
    for (auto& proto : fq) {
      std::vector<Predicate> pp;
      for (auto& pr : p.predicates)
        if (pr.protocol == proto && pr.is_binary()) {
          bool dup = false;
          for (auto& q : pp) dup = dup || q == pr;
          if (!dup) pp.push_back(pr);
        }
      std::sort(pp.begin(), pp.end());
      if (!lp.add_protocol(proto, pp)) throw FilterError("internal: add_protocol failed");
    }
    out.push_back(lp);
  }
  if (out.empty())
    throw FilterError("Invalid pattern. Contains unsupported layer encapsulation: " + p.str());
  std::sort(out.begin(), out.end(),
            [](const LayeredPattern& a, const LayeredPattern& b) { return a.to_flat() < b.to_flat(); });
  return out;
}

// ---------------------------------------------------------------------------------------------
// FlatPTree (ptree_flat.rs:80-267), only what Filter::new needs.
namespace {
struct FlatNode {
  Predicate pred;
  bool is_terminal = false;
  std::vector<FlatNode> children;
};

void flat_add(FlatNode& root, const FlatPattern& pattern) {
  FlatNode* node = &root;
  for (auto& pr : pattern.predicates) {
    FlatNode* next = nullptr;
    for (auto& c : node->children)
      if (c.pred == pr) { next = &c; break; }
    if (!next) {
      node->children.push_back(FlatNode{pr, false, {}});
      next = &node->children.back();
    }
    node = next;
  }
  node->is_terminal = true;
}

void flat_prune(FlatNode& n) {
  if (n.is_terminal) n.children.clear();
  for (auto& c : n.children) flat_prune(c);
}

void flat_patterns(const FlatNode& n, std::vector<Predicate>& preds, std::vector<FlatPattern>& out) {
  bool pushed = false;
  if (n.pred.protocol != "ethernet") {
    preds.push_back(n.pred);
    pushed = true;
  }
  if (n.is_terminal) {
    out.push_back(FlatPattern{preds});
  } else {
    for (auto& c : n.children) flat_patterns(c, preds, out);
  }
  if (pushed) preds.pop_back();
}
}  // namespace

// FlatPTree::new + prune_branches + to_flat_patterns (ptree_flat.rs:91-174, 257-267)
std::vector<FlatPattern> flat_ptree_pruned(const std::vector<FlatPattern>& patterns) {
  FlatNode root{Predicate::unary("ethernet"), false, {}};
  for (auto& f : patterns) flat_add(root, f);
  if (root.children.empty()) root.is_terminal = true;
  flat_prune(root);
  std::vector<FlatPattern> pruned;
  std::vector<Predicate> preds;
  flat_patterns(root, preds, pruned);
  return pruned;
}

// core/src/filter/mod.rs:113-139
Filter Filter::make(const std::string& filter_raw) {
  auto raw = parse_filter_raw(filter_raw);
  std::vector<LayeredPattern> fq;
  for (auto& r : raw) {
    auto v = to_fully_qualified(FlatPattern{r});
    fq.insert(fq.end(), v.begin(), v.end());
  }
  std::vector<FlatPattern> flat;
  for (auto& l : fq) flat.push_back(l.to_flat());
  std::sort(flat.begin(), flat.end());
  flat.erase(std::unique(flat.begin(), flat.end()), flat.end());

  auto pruned = flat_ptree_pruned(flat);
  Filter f;
  for (auto& p : pruned) {
    auto v = to_fully_qualified(p);
    f.patterns.insert(f.patterns.end(), v.begin(), v.end());
  }
  return f;
}

std::vector<FlatPattern> Filter::get_patterns_flat() const {
  std::vector<FlatPattern> v;
  for (auto& p : patterns) v.push_back(p.to_flat());
  return v;
}

// ---------------------------------------------------------------------------------------------
// Actions (Debug form used in PTree Display and in outcome_eq path strings)
std::string Actions::debug() const {
  static const char* names[] = {"PacketContinue", "PacketDeliver", "PacketCache", "PacketTrack", "ProtoProbe",
                                "ProtoFilter",    "SessionFilter", "SessionDeliver", "SessionTrack", "UpdatePDU",
                                "Reassemble",     "ConnDeliver",   "Stream"};
  auto one = [&](uint32_t bits) {
    std::string s = "[";
    bool first = true;
    for (int k = 0; k < 13; ++k)
      if (bits & (1u << k)) {
        if (!first) s += ", ";
        s += names[k];
        first = false;
      }
    return s + "]";
  };
  return "Actions { data: " + one(data) + ", terminal_actions: " + one(terminal) + " }";
}

const char* filter_layer_str(FilterLayer l) {
  switch (l) {
    case FilterLayer::PacketContinue: return "Pkt (pass)";
    case FilterLayer::Packet: return "Pkt";
    case FilterLayer::Protocol: return "Proto";
    case FilterLayer::Session: return "S";
    case FilterLayer::ConnectionDeliver: return "C (D)";
    case FilterLayer::PacketDeliver: return "Pkt (D)";
  }
  return "?";
}

// ---------------------------------------------------------------------------------------------
// DataType (datatypes.rs:100-397)
DataType DataType::connection(const std::string& n) {
  DataType d;
  d.level = Level::Connection;
  d.needs_update = true;
  d.as_str = n;
  return d;
}
DataType DataType::session(const std::string& n) {
  DataType d;
  d.level = Level::Session;
  d.needs_parse = true;
  d.as_str = n;
  return d;
}
DataType DataType::packet(const std::string& n) {
  DataType d;
  d.level = Level::Packet;
  d.as_str = n;
  return d;
}
DataType DataType::static_(const std::string& n) {
  DataType d;
  d.level = Level::Static;
  d.as_str = n;
  return d;
}
DataType DataType::pktlist(const std::string& n, bool reassembly) {
  DataType d;
  d.level = Level::Connection;
  d.needs_reassembly = reassembly;
  d.needs_packet_track = true;
  d.as_str = n;
  return d;
}

bool lookup_datatype(const std::string& name, DataType& out) {
  static const std::map<std::string, DataType> table = [] {
    std::map<std::string, DataType> t;
    for (auto n : {"ConnRecord", "ConnDuration", "PktCount", "ByteCount", "InterArrivals", "ConnHistory"})
      t[n] = DataType::connection(n);
    for (auto n : {"HttpTransaction", "DnsTransaction", "TlsHandshake", "QuicStream", "SshHandshake"})
      t[n] = DataType::session(n);
    t["ZcFrame"] = DataType::packet("ZcFrame");
    t["Payload"] = DataType::packet("Payload");
    DataType sl;
    sl.level = Level::Connection;
    sl.needs_parse = true;
    sl.track_sessions = true;
    sl.as_str = "SessionList";
    t["SessionList"] = sl;
    for (auto n : {"BidirZcPktStream", "OrigZcPktStream", "RespZcPktStream", "BidirPktStream", "OrigPktStream",
                   "RespPktStream"})
      t[n] = DataType::pktlist(n, false);
    for (auto n : {"OrigZcPktsReassembled", "RespZcPktsReassembled", "OrigPktsReassembled", "RespPktsReassembled"})
      t[n] = DataType::pktlist(n, true);
    for (auto n : {"CoreId", "FiveTuple", "EtherTCI", "EthAddr", "FilterStr"}) t[n] = DataType::static_(n);
    return t;
  }();
  auto it = table.find(name);
  if (it == table.end()) return false;
  out = it->second;
  return true;
}

bool DataType::should_deliver(FilterLayer l, const Predicate& p, Level sub_level) const {
  switch (level) {
    case Level::Packet:
      switch (l) {
        case FilterLayer::PacketContinue: return p.on_packet();
        case FilterLayer::Protocol: return p.on_proto();
        case FilterLayer::Session: return p.on_session();
        case FilterLayer::PacketDeliver: return true;
        default: return false;
      }
    case Level::Connection: return l == FilterLayer::ConnectionDeliver;
    case Level::Session: return l == FilterLayer::Session;
    case Level::Static:
      if (sub_level != Level::Static) return false;
      return p.on_packet() ? l == FilterLayer::Packet : l == FilterLayer::ConnectionDeliver;
    case Level::Streaming: throw FilterError("Datatypes should not be streaming");
  }
  return false;
}

bool DataType::can_deliver(FilterLayer l, const Predicate& p) const {
  switch (level) {
    case Level::Packet:
      if (l == FilterLayer::PacketContinue) return p.on_packet();
      if (l == FilterLayer::Protocol) return p.on_proto() || p.on_packet();
      return true;
    case Level::Connection: return l == FilterLayer::ConnectionDeliver;
    case Level::Session: return l == FilterLayer::Session || l == FilterLayer::ConnectionDeliver;
    case Level::Static: return true;
    case Level::Streaming: throw FilterError("Datatypes should not be streaming");
  }
  return false;
}

static bool can_stream(Level l) { return l == Level::Connection || l == Level::Packet; }

static void dt_needs_update(const DataType& d, MatchingActions& a) {
  using namespace action;
  if (d.needs_update) {
    a.if_matched.data |= UpdatePDU;
    a.if_matched.terminal |= UpdatePDU;
    a.if_matching.data |= UpdatePDU;
  }
  if (d.needs_reassembly) {
    a.if_matched.data |= Reassemble;
    a.if_matched.terminal |= Reassemble;
    a.if_matching.data |= Reassemble;
  }
  if (d.needs_packet_track) {
    a.if_matched.data |= PacketTrack;
    a.if_matched.terminal |= PacketTrack;
    a.if_matching.data |= PacketTrack;
  }
}

static void dt_track_sessions(const DataType& d, MatchingActions& a, Level sub) {
  if ((sub == Level::Connection || sub == Level::Streaming) && (d.level == Level::Session || d.needs_parse))
    a.if_matched.data |= action::SessionTrack;
}

static void dt_conn_deliver(Level sub, MatchingActions& a) {
  if (sub == Level::Connection) {
    a.if_matched.data |= action::ConnDeliver;
    a.if_matched.terminal |= action::ConnDeliver;
  }
}

static MatchingActions dt_packet_filter(const DataType& d, Level sub) {
  using namespace action;
  MatchingActions a;
  if (d.level == Level::Packet && sub == Level::Packet) a.if_matching.data |= PacketCache;
  dt_needs_update(d, a);
  dt_conn_deliver(sub, a);
  if (d.needs_parse) {
    a.if_matched.data |= ProtoProbe;
    a.if_matched.terminal |= ProtoProbe;
    if (sub == Level::Connection) {
      a.if_matched.data |= SessionTrack;
      a.if_matched.terminal |= SessionTrack;
    }
  }
  if (d.level == Level::Session && (sub == Level::Session || sub == Level::Streaming)) {
    a.if_matched.data |= SessionDeliver;
    a.if_matched.terminal |= SessionDeliver;
  }
  return a;
}

static MatchingActions dt_proto_filter(const DataType& d, Level sub) {
  using namespace action;
  MatchingActions a;
  if (d.level == Level::Packet) {
    a.if_matched.data |= PacketDeliver;
    a.if_matched.terminal |= PacketDeliver;
    a.if_matching.data |= PacketCache;
  }
  dt_needs_update(d, a);
  dt_track_sessions(d, a, sub);
  dt_conn_deliver(sub, a);
  if (d.level == Level::Session && (sub == Level::Session || sub == Level::Streaming))
    a.if_matched.data |= SessionDeliver;
  return a;
}

static MatchingActions dt_session_filter(const DataType& d, Level sub) {
  using namespace action;
  MatchingActions a;
  if (d.level == Level::Packet) {
    a.if_matched.data |= PacketDeliver;
    a.if_matched.terminal |= PacketDeliver;
  }
  dt_needs_update(d, a);
  dt_track_sessions(d, a, sub);
  dt_conn_deliver(sub, a);
  a.if_matching = Actions();
  return a;
}

// datatypes.rs:433-443, 507-512
void SubscriptionSpec::add_datatype(const DataType& d) {
  if (level != Level::Streaming && level != Level::Connection) {
    Level next = d.level;
    if (level == Level::Connection || next == Level::Connection) level = Level::Connection;
    else if (level == Level::Session || next == Level::Session) level = Level::Session;
    else if (level == Level::Packet || next == Level::Packet) level = Level::Packet;
  }
  datatypes.push_back(d);
}

// datatypes.rs:449-504 (asserts become FilterError)
void SubscriptionSpec::validate_spec() const {
  auto count = [&](Level l) {
    size_t c = 0;
    for (auto& d : datatypes) c += d.level == l;
    return c;
  };
  if (level == Level::Packet) {
    if (datatypes.size() > 1) {
      if (count(Level::Packet) != 1)
        throw FilterError("Must have one packet-level datatype in packet-level subscription");
      if (count(Level::Static) < datatypes.size() - 1)
        throw FilterError("Non-static datatype in packet-level subscription");
    }
  } else if (count(Level::Packet) != 0) {
    throw FilterError("Packet-level datatype in non-packet subscription");
  }
  if (level == Level::Streaming) {
    size_t c = 0;
    for (auto& d : datatypes) c += can_stream(d.level);
    if (c != 1) throw FilterError("Must have one streamable datatype in streaming subscription");
  }
  if (count(Level::Session) > 1) throw FilterError("Multiple session-level datatypes in subscription");
  // filtergen/src/data.rs:262-297: a packet-level callback takes only the packet datatype plus
  // FilterStr / CoreId; anything else is a compile-time panic in the reference.
  if (level == Level::Packet)
    for (auto& d : datatypes)
      if (d.level != Level::Packet && d.as_str != "FilterStr" && d.as_str != "CoreId")
        throw FilterError("Invalid datatype in packet callback: " + d.as_str);
}

std::string SubscriptionSpec::as_str() const {
  std::string s = callback + "(";
  for (size_t k = 0; k < datatypes.size(); ++k) {
    if (k) s += ", ";
    s += datatypes[k].as_str;
  }
  return s + ")";
}

bool SubscriptionSpec::has_datatype(const std::string& n) const {
  for (auto& d : datatypes)
    if (d.as_str == n) return true;
  return false;
}

bool SubscriptionSpec::should_deliver(FilterLayer l, const Predicate& p) const {
  if (level == Level::Streaming) return false;
  bool any = false, all = true;
  for (auto& d : datatypes) {
    any = any || d.should_deliver(l, p, level);
    all = all && d.can_deliver(l, p);
  }
  return any && all;
}

bool SubscriptionSpec::deliver_on_session() const {
  if (level == Level::Session) return true;
  if (level == Level::Streaming)
    for (auto& d : datatypes)
      if (d.level == Level::Session) return true;
  return false;
}

// ast.rs:151-184
bool SubscriptionSpec::pred_is_prev_layer(const Predicate& p, FilterLayer l) const {
  switch (l) {
    case FilterLayer::PacketContinue: return false;
    case FilterLayer::Packet: return p.on_packet() && level == Level::Packet;
    case FilterLayer::PacketDeliver: return level != Level::Packet || p.on_packet();
    case FilterLayer::Protocol: return p.on_packet();
    case FilterLayer::Session: return (p.on_packet() || p.on_proto()) && !deliver_on_session();
    case FilterLayer::ConnectionDeliver:
      return !(level == Level::Connection || level == Level::Static) || (level == Level::Static && p.on_packet());
  }
  return false;
}

// datatypes.rs:582-615
bool SubscriptionSpec::should_stream(FilterLayer l, const Predicate& p) const {
  if (level != Level::Streaming) return false;
  if (l == FilterLayer::PacketContinue) return false;
  for (auto& d : datatypes)
    if (!d.can_deliver(l, p) && !can_stream(d.level)) return false;
  bool all = true;
  for (auto& d : datatypes) all = all && (can_stream(d.level) || d.level == Level::Static);
  if (all) {
    if (l == FilterLayer::Packet) return p.on_packet();
    return !pred_is_prev_layer(p, l);
  }
  for (auto& d : datatypes)
    if (d.should_deliver(l, p, level)) return true;
  return false;
}

MatchingActions SubscriptionSpec::packet_continue() const {
  MatchingActions a;
  if (level == Level::Packet) {
    a.if_matching.data |= action::PacketContinue;
  } else {
    a.if_matched.data |= action::PacketContinue;
    a.if_matching.data |= action::PacketContinue;
  }
  return a;
}

MatchingActions SubscriptionSpec::packet_filter() const {
  MatchingActions a;
  for (auto& d : datatypes) {
    auto x = dt_packet_filter(d, level);
    a.if_matched.push(x.if_matched);
    a.if_matching.push(x.if_matching);
  }
  a.if_matching.data |= action::ProtoFilter;
  if (level == Level::Streaming) {
    a.if_matched.data |= action::Stream;
    a.if_matched.terminal |= action::Stream;
  }
  return a;
}

MatchingActions SubscriptionSpec::proto_filter() const {
  MatchingActions a;
  for (auto& d : datatypes) {
    auto x = dt_proto_filter(d, level);
    a.if_matched.push(x.if_matched);
    a.if_matching.push(x.if_matching);
  }
  if (level == Level::Static) {
    a.if_matched.data |= action::ConnDeliver;
    a.if_matched.terminal |= action::ConnDeliver;
  }
  if (level == Level::Streaming) {
    a.if_matched.data |= action::Stream;
    a.if_matched.terminal |= action::Stream;
  }
  a.if_matching.data |= action::SessionFilter;
  return a;
}

MatchingActions SubscriptionSpec::session_filter() const {
  MatchingActions a;
  for (auto& d : datatypes) {
    auto x = dt_session_filter(d, level);
    a.if_matched.push(x.if_matched);
    a.if_matching.push(x.if_matching);
  }
  if (level == Level::Static) {
    a.if_matched.data |= action::ConnDeliver;
    a.if_matched.terminal |= action::ConnDeliver;
  }
  if (level == Level::Streaming) {
    a.if_matched.data |= action::Stream;
    a.if_matched.terminal |= action::Stream;
  }
  return a;
}

Actions SubscriptionSpec::with_term_filter(FilterLayer l, const Predicate& p) const {
  switch (l) {
    case FilterLayer::PacketContinue: return packet_continue().if_matched;
    case FilterLayer::Packet: return packet_filter().if_matched;
    case FilterLayer::Protocol: return proto_filter().if_matched;
    case FilterLayer::Session: {
      Actions a = session_filter().if_matched;
      if (level == Level::Connection && p.on_session()) a.data |= action::SessionTrack;
      return a;
    }
    default: return Actions();
  }
}

Actions SubscriptionSpec::with_nonterm_filter(FilterLayer l) const {
  switch (l) {
    case FilterLayer::PacketContinue: return packet_continue().if_matching;
    case FilterLayer::Packet: return packet_filter().if_matching;
    case FilterLayer::Protocol: return proto_filter().if_matching;
    case FilterLayer::Session: return session_filter().if_matching;
    default: return Actions();
  }
}

SubscriptionSpec SubscriptionSpec::default_connection() {
  SubscriptionSpec s("fil", "cb");
  s.level = Level::Connection;
  s.datatypes.push_back(DataType::connection("Connection"));
  return s;
}
SubscriptionSpec SubscriptionSpec::default_session() {
  SubscriptionSpec s("fil", "cb");
  s.level = Level::Session;
  s.datatypes.push_back(DataType::session("Session"));
  return s;
}
SubscriptionSpec SubscriptionSpec::default_packet() {
  SubscriptionSpec s("fil", "cb");
  s.level = Level::Packet;
  s.datatypes.push_back(DataType::packet("Packet"));
  return s;
}
SubscriptionSpec SubscriptionSpec::default_streaming() {
  SubscriptionSpec s("fil", "cb");
  s.level = Level::Streaming;
  s.datatypes.push_back(DataType::connection("Connection"));
  return s;
}

// ---------------------------------------------------------------------------------------------
// Minimal TOML reader for subscription spec files (filtergen/src/parse.rs:7-66):
//   [[subscriptions]] tables with filter = "..", datatypes = ".." | [".."], callback = "..",
//   optional streaming = { seconds|packets|bytes = N } or streaming = "seconds=N".
namespace {
struct Toml {
  const std::string& s;
  size_t p = 0;
  size_t line = 1;
  explicit Toml(const std::string& t) : s(t) {}
  [[noreturn]] void fail(const std::string& m) {
    throw FilterError("ERROR: Config file invalid (line " + std::to_string(line) + "): " + m);
  }
  void skip_ws_comments(bool newlines) {
    while (p < s.size()) {
      char c = s[p];
      if (c == ' ' || c == '\t') { ++p; continue; }
      if (c == '#') { while (p < s.size() && s[p] != '\n') ++p; continue; }
      if (newlines && (c == '\n' || c == '\r')) { if (c == '\n') ++line; ++p; continue; }
      break;
    }
  }
  std::string key() {
    size_t b = p;
    while (p < s.size() && (isalnum((unsigned char)s[p]) || s[p] == '_' || s[p] == '-')) ++p;
    if (b == p) fail("expected key");
    return s.substr(b, p - b);
  }
  std::string str() {
    if (p >= s.size()) fail("expected string");
    char q = s[p];
    if (q != '"' && q != '\'') fail("expected string");
    bool multi = s.compare(p, 3, std::string(3, q)) == 0;
    std::string out;
    if (multi) {
      p += 3;
      if (p < s.size() && s[p] == '\n') { ++p; ++line; }
      while (p < s.size() && s.compare(p, 3, std::string(3, q)) != 0) {
        if (s[p] == '\n') ++line;
        if (q == '"' && s[p] == '\\') out += escape();
        else out += s[p++];
      }
      if (p >= s.size()) fail("unterminated string");
      p += 3;
      return out;
    }
    ++p;
    while (p < s.size() && s[p] != q) {
      if (s[p] == '\n') fail("newline in string");
      if (q == '"' && s[p] == '\\') out += escape();
      else out += s[p++];
    }
    if (p >= s.size()) fail("unterminated string");
    ++p;
    return out;
  }
  std::string escape() {
    ++p;
    if (p >= s.size()) fail("bad escape");
    char c = s[p++];
    switch (c) {
      case 'n': return "\n";
      case 't': return "\t";
      case 'r': return "\r";
      case '\\': return "\\";
      case '"': return "\"";
      case '\'': return "'";
      case 'u': {
        if (p + 4 > s.size()) fail("bad escape");
        unsigned v = std::stoul(s.substr(p, 4), nullptr, 16);
        p += 4;
        std::string o;
        if (v < 0x80) o += (char)v;
        else if (v < 0x800) { o += (char)(0xC0 | (v >> 6)); o += (char)(0x80 | (v & 63)); }
        else { o += (char)(0xE0 | (v >> 12)); o += (char)(0x80 | ((v >> 6) & 63)); o += (char)(0x80 | (v & 63)); }
        return o;
      }
      default: fail(std::string("bad escape \\") + c);
    }
  }
  double number() {
    size_t b = p;
    while (p < s.size() && (isdigit((unsigned char)s[p]) || s[p] == '.' || s[p] == '-' || s[p] == '+' ||
                            s[p] == 'e' || s[p] == 'E' || s[p] == '_'))
      ++p;
    if (b == p) fail("expected value");
    std::string t;
    for (size_t k = b; k < p; ++k)
      if (s[k] != '_') t += s[k];
    return std::stod(t);
  }
};
}  // namespace

std::vector<SubscriptionSpec> parse_subscription_toml(const std::string& text) {
  struct Raw {
    std::string filter, callback;
    std::vector<std::string> datatypes;
    bool has_filter = false, has_cb = false, has_dt = false, streaming = false;
  };
  std::vector<Raw> raws;
  Toml t(text);
  for (;;) {
    t.skip_ws_comments(true);
    if (t.p >= t.s.size()) break;
    if (t.s.compare(t.p, 2, "[[") == 0) {
      t.p += 2;
      t.skip_ws_comments(false);
      std::string k = t.key();
      t.skip_ws_comments(false);
      if (t.s.compare(t.p, 2, "]]") != 0) t.fail("expected ]]");
      t.p += 2;
      if (k != "subscriptions") t.fail("unknown table " + k);
      raws.emplace_back();
      continue;
    }
    std::string k = t.key();
    t.skip_ws_comments(false);
    if (t.p >= t.s.size() || t.s[t.p] != '=') t.fail("expected =");
    ++t.p;
    t.skip_ws_comments(false);
    if (raws.empty()) t.fail("key outside [[subscriptions]]");
    Raw& r = raws.back();
    if (k == "filter") {
      r.filter = t.str();
      r.has_filter = true;
    } else if (k == "callback") {
      r.callback = t.str();
      r.has_cb = true;
    } else if (k == "datatypes") {
      r.has_dt = true;
      if (t.s[t.p] == '[') {
        ++t.p;
        for (;;) {
          t.skip_ws_comments(true);
          if (t.p < t.s.size() && t.s[t.p] == ']') { ++t.p; break; }
          r.datatypes.push_back(t.str());
          t.skip_ws_comments(true);
          if (t.p < t.s.size() && t.s[t.p] == ',') { ++t.p; continue; }
          t.skip_ws_comments(true);
          if (t.p < t.s.size() && t.s[t.p] == ']') { ++t.p; break; }
          t.fail("expected , or ]");
        }
      } else {
        r.datatypes.push_back(t.str());
      }
    } else if (k == "streaming") {
      r.streaming = true;
      if (t.s[t.p] == '{') {
        ++t.p;
        t.skip_ws_comments(false);
        std::string sk = t.key();
        if (sk != "seconds" && sk != "packets" && sk != "bytes" && sk != "Seconds" && sk != "Packets" && sk != "Bytes")
          t.fail("Unknown Streaming variant: " + sk);
        t.skip_ws_comments(false);
        if (t.s[t.p] != '=') t.fail("expected =");
        ++t.p;
        t.skip_ws_comments(false);
        t.number();
        t.skip_ws_comments(false);
        if (t.s[t.p] != '}') t.fail("expected }");
        ++t.p;
      } else {
        t.str();
      }
    } else {
      t.fail("unknown key " + k);
    }
    t.skip_ws_comments(false);
    if (t.p < t.s.size() && t.s[t.p] != '\n' && t.s[t.p] != '\r') t.fail("trailing characters");
  }
  std::vector<SubscriptionSpec> out;
  for (auto& r : raws) {
    if (!r.has_filter || !r.has_cb || !r.has_dt) throw FilterError("ERROR: Config file invalid: missing field");
    if (r.datatypes.empty()) throw FilterError("subscription without datatypes");
    SubscriptionSpec spec(r.filter, r.callback);
    if (r.streaming) spec.level = Level::Streaming;
    for (auto& d : r.datatypes) {
      DataType dt;
      if (!lookup_datatype(d, dt)) throw FilterError("Invalid datatype: " + d);
      spec.add_datatype(dt);
    }
    spec.validate_spec();
    out.push_back(spec);
  }
  return out;
}

}  // namespace rtn
