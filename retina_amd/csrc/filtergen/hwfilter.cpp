// Hardware (NIC) filter rules. See hwfilter.hpp for the reference map.
#include "hwfilter.hpp"

#include <algorithm>
#include <climits>

namespace rtn {

namespace {

void put_be(uint8_t* p, uint64_t v, int bytes) {
  for (int k = bytes - 1; k >= 0; --k, v >>= 8) p[k] = uint8_t(v);
}

struct FieldSlot {
  const char* name;
  int offset, bytes;
};

// Field -> (offset, size) in the DPDK header struct the item carries (flow_item.rs:81-501).
// The names are the ones flow_item.rs matches on: "data_offset_to_nw" is not a filter field
// (the TCP accessor is data_offset_to_ns, tcp.rs:74-78), so that predicate never reaches the NIC.
const FieldSlot kIpv4[] = {{"version_ihl", 0, 1},    {"type_of_service", 1, 1},
                           {"total_length", 2, 2},   {"identification", 4, 2},
                           {"flags_to_fragment_offset", 6, 2}, {"time_to_live", 8, 1},
                           {"protocol", 9, 1},       {"header_checksum", 10, 2}};
const FieldSlot kIpv6[] = {{"version_to_flow_label", 0, 4}, {"payload_length", 4, 2},
                           {"next_header", 6, 1},           {"hop_limit", 7, 1}};
const FieldSlot kTcp[] = {{"src_port", 0, 2},          {"dst_port", 2, 2}, {"seq_no", 4, 4},
                          {"ack_no", 8, 4},            {"data_offset_to_nw", 12, 1},
                          {"flags", 13, 1},            {"window", 14, 2},  {"checksum", 16, 2},
                          {"urgent_pointer", 18, 2}};
const FieldSlot kUdp[] = {{"src_port", 0, 2}, {"dst_port", 2, 2}, {"length", 4, 2}, {"checksum", 6, 2}};

// One append_<proto> (flow_item.rs:81-500): every binary predicate of the layer writes its field
// (a later predicate on the same field overwrites); the operator is not looked at.
bool append_layer(const std::string& proto, const std::vector<Predicate>& preds, FlowItem& it,
                  std::string* why) {
  const FieldSlot* table = nullptr;
  size_t nt = 0;
  if (proto == "ipv4") {
    it.type = FLOW_IPV4, it.size = 20, table = kIpv4, nt = sizeof(kIpv4) / sizeof(kIpv4[0]);
  } else if (proto == "ipv6") {
    it.type = FLOW_IPV6, it.size = 40, table = kIpv6, nt = sizeof(kIpv6) / sizeof(kIpv6[0]);
  } else if (proto == "tcp") {
    it.type = FLOW_TCP, it.size = 20, table = kTcp, nt = sizeof(kTcp) / sizeof(kTcp[0]);
  } else if (proto == "udp") {
    it.type = FLOW_UDP, it.size = 8, table = kUdp, nt = sizeof(kUdp) / sizeof(kUdp[0]);
  } else {
    if (why) *why = "Invalid header: " + proto;  // FilterError::InvalidHeader
    return false;
  }
  for (auto& p : preds) {
    if (p.is_unary()) {
      if (why) *why = "Invalid predicate type: unary";
      return false;
    }
    const Value& v = p.value;
    // address fields take an IP network: spec = the address as written, mask = its netmask
    if ((proto == "ipv4" || proto == "ipv6") && (p.field == "src_addr" || p.field == "dst_addr")) {
      const int off = proto == "ipv4" ? (p.field == "src_addr" ? 12 : 16) : (p.field == "src_addr" ? 8 : 24);
      if (proto == "ipv4" && v.kind == VKind::Ipv4) {
        put_be(it.spec + off, v.v4.addr, 4);
        put_be(it.mask + off, v.v4.netmask(), 4);
        continue;
      }
      if (proto == "ipv6" && v.kind == VKind::Ipv6) {
        const U128 m = v.v6.netmask();
        put_be(it.spec + off, v.v6.addr.hi, 8);
        put_be(it.spec + off + 8, v.v6.addr.lo, 8);
        put_be(it.mask + off, m.hi, 8);
        put_be(it.mask + off + 8, m.lo, 8);
        continue;
      }
      if (why) *why = "Invalid RHS type: " + v.str();
      return false;
    }
    const FieldSlot* s = nullptr;
    for (size_t k = 0; k < nt && !s; ++k)
      if (p.field == table[k].name) s = &table[k];
    if (!s) {
      if (why) *why = "Invalid field: " + p.field;
      return false;
    }
    if (v.kind != VKind::Int) {
      if (why) *why = "Invalid RHS type: " + v.str();
      return false;
    }
    const uint64_t lim = s->bytes == 1 ? 0xFFull : s->bytes == 2 ? 0xFFFFull : 0xFFFFFFFFull;
    if (v.i > lim) {  // uN::try_from
      if (why) *why = "Invalid RHS value: " + v.str();
      return false;
    }
    put_be(it.spec + s->offset, v.i, s->bytes);
    put_be(it.mask + s->offset, lim, s->bytes);
  }
  return true;
}

FlowItem bare(uint32_t type) {
  FlowItem it;
  it.type = type;
  return it;
}

// pattern.rs:28-49
bool is_fully_qualified(const FlatPattern& f) {
  int prev = layer_index("ethernet");
  bool ret = true;
  for (auto& p : f.predicates) {
    const int cur = layer_index(p.protocol);
    if (cur < 0) return false;
    if (p.is_unary()) {
      ret = ret && layer_edge(cur, prev);
      prev = cur;
    } else {
      ret = ret && cur == prev;
    }
  }
  return ret;
}

// pattern_supported (hardware/mod.rs:185-203): a fully-qualified pattern is supported if it
// translates and the device validates it as a group-0, high-priority RSS rule.
bool pattern_supported(const LayeredPattern& lp, const FlowValidate& validate) {
  FlowRule r;
  r.group = 0, r.priority = kHwHighPriority, r.action = FLOW_ACTION_RSS;
  r.items.push_back(bare(FLOW_ETH));
  for (auto& layer : lp.layers) {
    FlowItem it;
    if (!append_layer(layer.first, layer.second, it, nullptr)) return false;
    r.items.push_back(it);
  }
  r.items.push_back(bare(FLOW_END));
  return !validate || validate(r);
}

// device_supported (hardware/mod.rs:124-173)
bool device_supported(const Predicate& p, const FlowValidate& validate) {
  static const char* kProtos[] = {"ipv4", "ipv6", "tcp", "udp"};
  if (std::none_of(std::begin(kProtos), std::end(kProtos), [&](const char* s) { return p.protocol == s; }))
    return false;
  if (p.is_binary()) {
    const bool ip = p.protocol == "ipv4" || p.protocol == "ipv6";
    if (!(p.op == BinOp::Eq || (ip && p.op == BinOp::In))) return false;
  }
  // predicate_supported (:175-183): every fully-qualified form of the lone predicate
  for (auto& lp : to_fully_qualified(FlatPattern{{p}}))
    if (!pattern_supported(lp, validate)) return false;
  return true;
}

}  // namespace

bool flow_items_from_layered(const LayeredPattern& lp, std::vector<FlowItem>& items, std::string* why) {
  items.clear();
  for (auto& layer : lp.layers) {
    FlowItem it;
    if (!append_layer(layer.first, layer.second, it, why)) return false;
    items.push_back(it);
  }
  return true;
}

HardwareFilter HardwareFilter::make(const Filter& filter, const FlowValidate& validate) {
  // retain_hardware_predicates (pattern.rs:133-142)
  std::vector<FlatPattern> hw;
  for (auto& f : filter.get_patterns_flat()) {
    FlatPattern kept;
    for (auto& p : f.predicates)
      if (device_supported(p, validate)) kept.predicates.push_back(p);
    hw.push_back(kept);
  }
  HardwareFilter out;
  for (auto& f : flat_ptree_pruned(hw)) {
    FlatPattern pat = f;
    while (!is_fully_qualified(pat)) pat.predicates.pop_back();  // broaden
    for (auto& lp : to_fully_qualified(pat)) out.patterns.push_back(lp);
  }
  auto by_flat = [](const LayeredPattern& a, const LayeredPattern& b) { return a.to_flat() < b.to_flat(); };
  std::sort(out.patterns.begin(), out.patterns.end(), by_flat);
  out.patterns.erase(std::unique(out.patterns.begin(), out.patterns.end(),
                                 [](const LayeredPattern& a, const LayeredPattern& b) {
                                   return a.to_flat() == b.to_flat();
                                 }),
                     out.patterns.end());
  return out;
}

std::vector<FlowRule> HardwareFilter::rules() const {
  std::vector<FlowRule> out;
  if (std::all_of(patterns.begin(), patterns.end(), [](const LayeredPattern& p) { return p.layers.empty(); }))
    return out;
  for (size_t k = 0; k < patterns.size(); ++k) {
    FlowRule r;
    r.group = 0, r.priority = kHwHighPriority, r.action = FLOW_ACTION_RSS, r.pattern = uint32_t(k);
    std::vector<FlowItem> items;
    std::string why;
    if (!flow_items_from_layered(patterns[k], items, &why))  // HardwareFilterError::InvalidRule
      throw FilterError("Hardware flow rule invalid: " + patterns[k].to_flat().str() + " (" + why + ")");
    r.items.push_back(bare(FLOW_ETH));
    r.items.insert(r.items.end(), items.begin(), items.end());
    r.items.push_back(bare(FLOW_END));
    out.push_back(r);
  }
  // add_redirect (hardware/mod.rs:332-392): everything else jumps to group 1, where it is dropped
  FlowRule j;
  j.group = 0, j.priority = kHwLowPriority, j.action = FLOW_ACTION_JUMP, j.jump_group = 1;
  j.pattern = UINT32_MAX;
  j.items = {bare(FLOW_ETH), bare(FLOW_END)};
  out.push_back(j);
  return out;
}

std::string HardwareFilter::str() const {
  std::string s;
  for (auto& p : patterns) s += p.to_flat().str() + "\n";
  return s;
}

}  // namespace rtn
