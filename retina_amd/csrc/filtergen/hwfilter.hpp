// Hardware (NIC) filter: the rte_flow rules Retina installs for a filter.
//
// Reference map (stanford-esrg/retina):
//   core/src/filter/hardware/mod.rs:35-73     HardwareFilter::new (retain device-supported
//                                             predicates, FlatPTree prune, broaden until fully
//                                             qualified, to_fully_qualified, sort + dedup)
//   core/src/filter/hardware/mod.rs:76-93     install: one rule per pattern (group 0, priority 0,
//                                             RSS), then the group 0 -> 1 jump (priority 3)
//   core/src/filter/hardware/mod.rs:124-203   device_supported / predicate_supported /
//                                             pattern_supported (rte_flow_validate per
//                                             fully-qualified single-predicate pattern)
//   core/src/filter/hardware/flow_item.rs:49-501  FlowPattern::from_layered_pattern: ETH, then one
//                                             item per layer with spec/mask in DPDK's rte_*_hdr
//                                             byte layout (wire order), then END
//   core/src/filter/pattern.rs:28-49, 133-142 is_fully_qualified / retain_hardware_predicates
// The device check (rte_flow_validate on a port) is a caller-supplied function: this code has no
// NIC, so whatever a port accepts is the caller's to say.
#pragma once

#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "filter.hpp"

namespace rtn {

enum FlowItemType : uint32_t { FLOW_END = 0, FLOW_ETH = 1, FLOW_IPV4 = 2, FLOW_IPV6 = 3, FLOW_TCP = 4, FLOW_UDP = 5 };
enum FlowActionType : uint32_t { FLOW_ACTION_RSS = 1, FLOW_ACTION_JUMP = 2 };

struct FlowItem {
  uint32_t type = FLOW_END;
  uint32_t size = 0;  // bytes of spec/mask that hold the header (rte_ipv4_hdr 20, rte_ipv6_hdr 40, ...)
  uint8_t spec[40] = {};
  uint8_t mask[40] = {};
};

struct FlowRule {
  uint32_t group = 0, priority = 0;
  uint32_t action = FLOW_ACTION_RSS;
  uint32_t jump_group = 0;
  uint32_t pattern = 0;        // index into HardwareFilter::patterns, UINT32_MAX for the redirect
  std::vector<FlowItem> items;  // ETH ... END
};

// rte_flow_validate(port, attr, pattern, RSS action) == 0
using FlowValidate = std::function<bool(const FlowRule&)>;

constexpr uint32_t kHwHighPriority = 0;  // hardware/mod.rs:26
constexpr uint32_t kHwLowPriority = 3;   // hardware/mod.rs:27

// FlowPattern::from_layered_pattern (flow_item.rs:66-79). Returns false and a reason (the
// FilterError the reference bails with) when a layer, field or value has no rte_flow form.
bool flow_items_from_layered(const LayeredPattern& lp, std::vector<FlowItem>& items, std::string* why);

struct HardwareFilter {
  std::vector<LayeredPattern> patterns;
  // HardwareFilter::new (hardware/mod.rs:38-73) for Filter::new(filter_str).
  static HardwareFilter make(const Filter& filter, const FlowValidate& validate);
  // The rules install() creates, in order (hardware/mod.rs:76-93); empty when the filter is
  // empty ("Empty filter, skipping.").
  std::vector<FlowRule> rules() const;
  std::string str() const;  // Display: one flat pattern per line
};

}  // namespace rtn
