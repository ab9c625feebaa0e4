/*
 * retina_hw.h — the NIC-side (hardware-assist) filter as rte_flow rules.
 *
 * With `online.hardware_assist` (core/src/config.rs:327-328), Retina parses the program's
 * hardware filter string (FilterFactory.filter_str, get_hw_filter in filtergen/src/lib.rs:233-238;
 * rtn_program_hw_filter) with Filter::new (core/src/runtime/online.rs:39) and installs it on every
 * port (Filter::set_hardware_filter, core/src/filter/mod.rs:165-174):
 *   - HardwareFilter::new (core/src/filter/hardware/mod.rs:38-73) keeps each pattern's predicates
 *     that the device supports (device_supported, :124-173: ipv4/ipv6/tcp/udp, `=` or an IP `in`,
 *     and rte_flow_validate accepts every fully-qualified form of the lone predicate), prunes the
 *     patterns (FlatPTree), broadens each until it is fully qualified, then sorts and dedups them;
 *   - install (:76-93) creates one rule per pattern on group 0 at priority 0 with an RSS action
 *     (pattern ETH, one item per layer with spec/mask from FlowPattern::from_layered_pattern,
 *     hardware/flow_item.rs:66-501, END), then a group-0 -> group-1 JUMP rule at priority 3 for
 *     everything else (add_redirect, :332-392). An empty filter installs nothing.
 * This library produces those rules; creating them is the caller's rte_flow_create (there is no
 * DPDK here). If any creation fails the reference flushes the port's rules and passes all traffic
 * (core/src/runtime/online.rs:184-191, hardware/mod.rs:453-466): callers should do the same.
 *
 * Item specs and masks are the bytes of DPDK's header structs (struct rte_ipv4_hdr, rte_ipv6_hdr,
 * rte_tcp_hdr, rte_udp_hdr), which are wire order: they can be memcpy'd into the
 * rte_flow_item_{ipv4,ipv6,tcp,udp}.hdr the item points at. The RSS action's queues are the port's
 * RETA (hardware/mod.rs:222-231), which the caller owns.
 */
#ifndef RETINA_HW_H
#define RETINA_HW_H

#include <stddef.h>
#include <stdint.h>

#include "retina_pc.h"

#ifdef __cplusplus
extern "C" {
#endif

/* rtn_flow_item_t.type (item_type; map to RTE_FLOW_ITEM_TYPE_*) */
#define RTN_FLOW_ITEM_END 0u
#define RTN_FLOW_ITEM_ETH 1u  /* no spec/mask: any Ethernet frame                   */
#define RTN_FLOW_ITEM_IPV4 2u /* 20 bytes: struct rte_ipv4_hdr                      */
#define RTN_FLOW_ITEM_IPV6 3u /* 40 bytes: struct rte_ipv6_hdr                      */
#define RTN_FLOW_ITEM_TCP 4u  /* 20 bytes: struct rte_tcp_hdr                       */
#define RTN_FLOW_ITEM_UDP 5u  /* 8 bytes: struct rte_udp_hdr                        */

/* rtn_flow_rule_t.action (map to RTE_FLOW_ACTION_TYPE_*, followed by END) */
#define RTN_FLOW_ACTION_RSS 1u  /* RSS over the port's RETA queues                 */
#define RTN_FLOW_ACTION_JUMP 2u /* jump to jump_group                              */

#define RTN_FLOW_MAX_ITEMS 4u /* ETH, L3, L4, END                                  */
#define RTN_FLOW_REDIRECT 0xFFFFFFFFu

typedef struct rtn_flow_item {
  uint32_t item_type; /* RTN_FLOW_ITEM_*                                    */
  uint32_t size; /* bytes of spec/mask in use (0 for ETH and END)           */
  uint8_t spec[40];
  uint8_t mask[40]; /* 0xFF bytes on every matched field; netmask for addresses */
} rtn_flow_item_t;

typedef struct rtn_flow_rule {
  uint32_t group;      /* rte_flow_attr.group (ingress)                        */
  uint32_t priority;   /* rte_flow_attr.priority: 0 for patterns, 3 for the jump */
  uint32_t action;     /* RTN_FLOW_ACTION_*                                    */
  uint32_t jump_group; /* RTN_FLOW_ACTION_JUMP only                            */
  uint32_t pattern;    /* line of rtn_hw_patterns, RTN_FLOW_REDIRECT for the jump */
  uint32_t n_items;    /* items in use, ETH first and END last                 */
  rtn_flow_item_t items[RTN_FLOW_MAX_ITEMS];
} rtn_flow_rule_t;

/* The device check: return nonzero if the port accepts `rule` (rte_flow_validate(port, attr,
 * pattern, RSS action) == 0). Called with group-0, priority-0 RSS rules, once per fully-qualified
 * form of each candidate predicate; it must be a pure function of the rule. NULL: the device
 * accepts every rule this translation can express. */
typedef int32_t (*rtn_flow_validate_fn)(void* user, const rtn_flow_rule_t* rule);

/* The rules installed for `filter` (a filter string, parsed as Filter::new does). Writes at most
 * cap rules and sets *n_rules to the number there are (patterns + 1, or 0 for an empty filter):
 * RTN_ERANGE if cap is smaller, RTN_EFILTER if the string is not a valid filter. */
int32_t rtn_hw_rules(const char* filter, rtn_flow_validate_fn validate, void* user,
                     rtn_flow_rule_t* rules, uint32_t cap, uint32_t* n_rules);
/* The same for a compiled program's hardware filter string (rtn_program_hw_filter). */
int32_t rtn_program_hw_rules(const rtn_program_t* p, rtn_flow_validate_fn validate, void* user,
                             rtn_flow_rule_t* rules, uint32_t cap, uint32_t* n_rules);
/* HardwareFilter's Display: its patterns, one flat pattern per line (rule k's line is k).
 * Returns the length needed; copies at most cap-1 bytes + NUL (0 and an error on failure). */
size_t rtn_hw_patterns(const char* filter, rtn_flow_validate_fn validate, void* user, char* buf,
                       size_t cap);

#ifdef __cplusplus
}
#endif

#endif /* RETINA_HW_H */
