// C ABI of the hardware-assist filter (include/retina_hw.h): the rte_flow rules Retina's
// Filter::set_hardware_filter installs (core/src/filter/hardware/mod.rs:38-93), as plain structs.
#include "retina_hw.h"

#include <cstring>
#include <string>

#include "../filtergen/hwfilter.hpp"
#include "rtn_error.hpp"

namespace {

void to_c(const rtn::FlowRule& r, rtn_flow_rule_t& o) {
  memset(&o, 0, sizeof(o));
  o.group = r.group;
  o.priority = r.priority;
  o.action = r.action;
  o.jump_group = r.jump_group;
  o.pattern = r.pattern;
  o.n_items = uint32_t(r.items.size());
  for (size_t k = 0; k < r.items.size() && k < RTN_FLOW_MAX_ITEMS; ++k) {
    o.items[k].item_type = r.items[k].type;
    o.items[k].size = r.items[k].size;
    memcpy(o.items[k].spec, r.items[k].spec, sizeof(o.items[k].spec));
    memcpy(o.items[k].mask, r.items[k].mask, sizeof(o.items[k].mask));
  }
}

rtn::FlowValidate wrap(rtn_flow_validate_fn fn, void* user) {
  if (!fn) return nullptr;
  return [fn, user](const rtn::FlowRule& r) {
    rtn_flow_rule_t c;
    to_c(r, c);
    return fn(user, &c) != 0;
  };
}

// Filter::new(filter_str) then HardwareFilter::new (core/src/runtime/online.rs:39,
// core/src/filter/mod.rs:165-167)
int32_t make(const char* filter, rtn_flow_validate_fn fn, void* user, rtn::HardwareFilter& out) {
  if (!filter) return rtn::set_error(RTN_EINVAL, "null filter");
  try {
    out = rtn::HardwareFilter::make(rtn::Filter::make(filter), wrap(fn, user));
    return RTN_OK;
  } catch (const rtn::FilterError& e) {
    return rtn::set_error(RTN_EFILTER, e.what());
  } catch (const std::exception& e) {
    return rtn::set_error(RTN_EFILTER, std::string("internal error: ") + e.what());
  }
}

}  // namespace

extern "C" {

int32_t rtn_hw_rules(const char* filter, rtn_flow_validate_fn validate, void* user, rtn_flow_rule_t* rules,
                     uint32_t cap, uint32_t* n_rules) {
  if (!n_rules || (cap && !rules)) return rtn::set_error(RTN_EINVAL, "null argument");
  rtn::HardwareFilter hw;
  int32_t rc = make(filter, validate, user, hw);
  if (rc != RTN_OK) return rc;
  std::vector<rtn::FlowRule> rs;
  try {
    rs = hw.rules();
  } catch (const rtn::FilterError& e) {
    return rtn::set_error(RTN_EFILTER, e.what());
  }
  *n_rules = uint32_t(rs.size());
  if (rs.size() > cap) return rtn::set_error(RTN_ERANGE, "rule buffer too small");
  for (size_t k = 0; k < rs.size(); ++k) to_c(rs[k], rules[k]);
  return RTN_OK;
}

size_t rtn_hw_patterns(const char* filter, rtn_flow_validate_fn validate, void* user, char* buf, size_t cap) {
  rtn::HardwareFilter hw;
  if (make(filter, validate, user, hw) != RTN_OK) {
    if (buf && cap) buf[0] = 0;
    return 0;
  }
  const std::string s = hw.str();
  if (buf && cap > 0) {
    size_t n = s.size() < cap - 1 ? s.size() : cap - 1;
    memcpy(buf, s.data(), n);
    buf[n] = 0;
  }
  return s.size();
}

}  // extern "C"
