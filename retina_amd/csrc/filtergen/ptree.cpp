// Predicate tree construction and collapse: a restatement of core/src/filter/ptree.rs.
// Line references are to that file unless stated.
#include <algorithm>
#include <functional>

#include "filter.hpp"

namespace rtn {

// PNode Display (246-274). The deliver set prints in ascending subscription id.
std::string PNode::display() const {
  std::string s = pred.str();
  if (!actions.drop()) s += " -- A: " + actions.debug();
  if (!deliver.empty()) {
    s += " D: ( ";
    for (auto& d : deliver) s += d.as_str + ", ";
    s += ")";
  }
  if (!stream.empty()) {
    s += " Stream (start): ( ";
    for (auto& d : stream) s += d.as_str + ", ";
    s += ")";
  }
  if (if_else) s += " x";
  return s;
}

namespace {

bool has_descendant(const PNode& n, const Predicate& pred) {
  for (auto& c : n.children) {
    if (c.pred == pred) return true;
    if (pred.is_child(c.pred) && has_descendant(c, pred)) return true;
  }
  return false;
}

PNode* get_descendant(PNode& n, const Predicate& pred) {
  for (auto& c : n.children) {
    if (c.pred == pred) return &c;
    if (pred.is_child(c.pred)) {
      if (PNode* r = get_descendant(c, pred)) return r;
    }
  }
  return nullptr;
}

bool has_child(const PNode& n, const Predicate& pred) {
  for (auto& c : n.children)
    if (c.pred == pred) return true;
  return false;
}

PNode* get_child(PNode& n, const Predicate& pred) {
  for (auto& c : n.children)
    if (c.pred == pred) return &c;
  return nullptr;
}

bool has_children_of(const PNode& n, const Predicate& pred) {
  for (auto& c : n.children)
    if (c.pred.is_child(pred)) return true;
  return false;
}

std::vector<PNode> get_children_of(PNode& n, const Predicate& pred) {
  std::vector<PNode> moved, kept;
  for (auto& c : n.children) (c.pred.is_child(pred) ? moved : kept).push_back(std::move(c));
  n.children = std::move(kept);
  return moved;
}

PNode* get_parent_candidate(PNode& n, const Predicate& pred) {
  for (auto& c : n.children)
    if (pred.is_child(c.pred)) return &c;
  return nullptr;
}

bool has_parent(const PNode& n, const Predicate& pred) {
  for (auto& c : n.children)
    if (pred.is_child(c.pred)) return true;
  return false;
}

// 186-201: the most narrow parent
PNode* get_parent(PNode& start, const Predicate& pred, size_t tree_size) {
  PNode* node = &start;
  for (size_t k = 0; k < tree_size; ++k) {
    PNode* next = get_parent_candidate(*node, pred);
    if (!next) return nullptr;
    if (!get_parent_candidate(*next, pred)) return next;
    node = next;
  }
  return nullptr;
}

bool extracts_protocol(const PNode& n, FilterLayer layer) {
  if ((layer == FilterLayer::PacketDeliver || layer == FilterLayer::Packet) && n.pred.is_unary()) {
    for (auto& c : n.children)
      if (c.pred.is_unary()) return true;
  }
  if (!n.pred.is_unary()) return false;
  for (auto& c : n.children)
    if (n.pred.protocol == c.pred.protocol && c.pred.is_binary()) return true;
  return false;
}

void get_paths(const PNode& n, std::vector<std::string>& curr, std::vector<std::string>& paths) {
  if (n.children.empty() && !curr.empty()) {
    std::string j;
    for (size_t k = 0; k < curr.size(); ++k) {
      if (k) j += ",";
      j += curr[k];
    }
    paths.push_back(j);
  } else {
    for (auto& c : n.children) {
      curr.push_back(c.display());
      get_paths(c, curr, paths);
    }
  }
  if (!curr.empty()) curr.pop_back();
}

bool all_paths_eq(const PNode& a, const PNode& b) {
  if (a.children.empty() && b.children.empty()) return true;
  std::vector<std::string> pa, pb, cur;
  get_paths(a, cur, pa);
  cur.clear();
  get_paths(b, cur, pb);
  return pa == pb;
}

bool outcome_eq(const PNode& a, const PNode& b) {
  if (a.actions != b.actions || a.deliver != b.deliver) return false;
  return (a.children.empty() && b.children.empty()) || all_paths_eq(a, b);
}

bool is_prev_layer_pred(const Predicate& p, FilterLayer l) {
  switch (l) {
    case FilterLayer::PacketContinue: return false;
    case FilterLayer::Packet:
    case FilterLayer::Protocol: return p.on_packet();
    case FilterLayer::PacketDeliver:
    case FilterLayer::ConnectionDeliver: return true;
    case FilterLayer::Session: return p.on_packet() || p.on_proto();
  }
  return false;
}

bool is_next_layer(const Predicate& p, FilterLayer l) {
  switch (l) {
    case FilterLayer::Packet:
    case FilterLayer::PacketContinue: return !p.on_packet();
    case FilterLayer::Protocol: return p.on_session();
    default: return false;
  }
}

// Ord for PNode (898-927)
bool pnode_less(const PNode& a, const PNode& b) {
  if (a.pred.is_binary() && b.pred.is_binary() && a.pred.protocol == b.pred.protocol)
    return a.pred.field < b.pred.field;
  return a.pred.protocol < b.pred.protocol;
}

// Rust's slice::sort (stable): insertion sort up to 20 elements, a stable merge otherwise.
void rust_stable_sort(std::vector<PNode>& v) {
  if (v.size() <= 20) {
    for (size_t i = 1; i < v.size(); ++i) {
      size_t j = i;
      while (j > 0 && pnode_less(v[i], v[j - 1])) --j;
      if (j != i) {
        PNode tmp = std::move(v[i]);
        for (size_t k = i; k > j; --k) v[k] = std::move(v[k - 1]);
        v[j] = std::move(tmp);
      }
    }
    return;
  }
  std::stable_sort(v.begin(), v.end(), pnode_less);
}

bool windows_all_excl(const std::vector<PNode>& c) {
  for (size_t k = 1; k < c.size(); ++k)
    if (!c[k - 1].pred.is_excl(c[k].pred)) return false;
  return true;
}

}  // namespace

PTree::PTree(FilterLayer l) : layer(l) {
  root.pred = Predicate::unary("ethernet");
  root.id = 0;
}

void PTree::clear() {
  root = PNode();
  root.pred = Predicate::unary("ethernet");
  size = 1;
  actions = Actions();
  collapsed = false;
}

// 321-341
void PTree::add_filter(const std::vector<FlatPattern>& patterns, const SubscriptionSpec& sub, const Deliver& d) {
  if (collapsed) throw FilterError("Cannot add filter to tree after collapsing");
  if (layer == FilterLayer::PacketDeliver && sub.level != Level::Packet) return;
  if (layer == FilterLayer::ConnectionDeliver && !(sub.level == Level::Connection || sub.level == Level::Static))
    return;
  build_tree(patterns, sub, d);
}

// 344-385
void PTree::build_tree(const std::vector<FlatPattern>& patterns, const SubscriptionSpec& sub, const Deliver& d) {
  bool added = false;
  for (size_t i = 0; i < patterns.size(); ++i) {
    const auto& pat = patterns[i];
    bool prev = true;
    for (auto& p : pat.predicates) prev = prev && sub.pred_is_prev_layer(p, layer);
    if (prev) continue;
    added = added || !pat.predicates.empty();
    add_pattern(pat, i, sub, d);
  }
  if (!added && sub.pred_is_prev_layer(root.pred, layer) && !sub.should_stream(layer, root.pred)) return;
  if (!added) {
    Predicate pred = Predicate::unary("ethernet");
    if (sub.should_deliver(layer, pred)) {
      root.deliver.insert(d);
    } else if (sub.should_stream(layer, root.pred)) {
      root.stream.insert(d);
    } else {
      Actions a = sub.with_term_filter(layer, pred);
      root.actions.push(a);
      actions.push(a);
    }
  }
}

// 389-461
void PTree::add_pattern(const FlatPattern& pattern, size_t pattern_id, const SubscriptionSpec& sub, const Deliver& d) {
  PNode* node = &root;
  node->patterns.push_back(pattern_id);
  for (auto& predicate : pattern.predicates) {
    if (is_next_layer(predicate, layer)) {
      Actions a = sub.with_nonterm_filter(layer);
      node->actions.push(a);
      actions.push(a);
      return;
    }
    if (layer != FilterLayer::PacketContinue && predicate.req_packet())
      throw FilterError(
          "Cannot access per-packet fields (e.g., TCP flags, length) after packet filter.\n"
          "Subscribe to `ZcFrame` or list of mbufs instead.");
    if (has_descendant(*node, predicate)) {
      node = get_descendant(*node, predicate);
      node->patterns.push_back(pattern_id);
      continue;
    }
    if (has_parent(*node, predicate)) node = get_parent(*node, predicate, size);
    std::vector<PNode> kids;
    if (has_children_of(*node, predicate)) kids = get_children_of(*node, predicate);
    if (!has_child(*node, predicate)) {
      PNode n;
      n.pred = predicate;
      n.id = size;
      node->children.push_back(std::move(n));
      size += 1;
    }
    node = get_child(*node, predicate);
    for (auto& k : kids) node->children.push_back(std::move(k));
    node->patterns.push_back(pattern_id);
  }
  if (sub.should_deliver(layer, node->pred)) {
    node->deliver.insert(d);
  } else if (sub.should_stream(layer, node->pred)) {
    node->stream.insert(d);
  }
  Actions a = sub.with_term_filter(layer, node->pred);
  if (!a.drop()) {
    node->actions.push(a);
    actions.push(a);
  }
}

const PNode* PTree::get_subtree(size_t id) const {
  std::function<const PNode*(const PNode&)> f = [&](const PNode& n) -> const PNode* {
    if (n.id == id) return &n;
    for (auto& c : n.children)
      if (auto r = f(c)) return r;
    return nullptr;
  };
  return f(root);
}

void PTree::sort() {
  std::function<void(PNode&)> f = [&](PNode& n) {
    for (auto& c : n.children) f(c);
    rust_stable_sort(n.children);
  };
  f(root);
}

bool PTree::get_single_callback(Deliver& out) const {
  DeliverSet cbs;
  std::function<void(const PNode&)> f = [&](const PNode& n) {
    if (!n.deliver.empty()) cbs.insert(n.deliver.begin(), n.deliver.end());
    if (cbs.size() > 1) return;
    for (auto& c : n.children) f(c);
  };
  f(root);
  if (cbs.size() != 1) return false;
  out = *cbs.begin();
  return true;
}

// 527-552
void PTree::mark_mutual_exclusion() {
  std::function<void(PNode&)> f = [&](PNode& n) {
    for (size_t idx = 0; idx < n.children.size(); ++idx) {
      f(n.children[idx]);
      if (idx == 0) continue;
      if (n.children[idx].pred.is_excl(n.children[idx - 1].pred)) n.children[idx].if_else = true;
      if (outcome_eq(n.children[idx], n.children[idx - 1])) n.children[idx].if_else = true;
    }
  };
  f(root);
}

void PTree::update_size() {
  size_t id = 0;
  std::function<size_t(PNode&)> f = [&](PNode& n) -> size_t {
    n.id = id++;
    size_t c = 1;
    for (auto& k : n.children) c += f(k);
    return c;
  };
  size = f(root);
}

// 570-634
void PTree::prune_branches() {
  std::function<void(PNode&, const Actions&, const std::set<std::string>&, const std::set<std::string>&)> f =
      [&](PNode& n, const Actions& on_a, const std::set<std::string>& on_d, const std::set<std::string>& on_s) {
        std::set<std::string> my_d = on_d;
        DeliverSet nd;
        for (auto& i : n.deliver) {
          if (!my_d.count(i.as_str)) {
            my_d.insert(i.as_str);
            nd.insert(i);
          } else if (i.must_deliver) {
            nd.insert(i);
          }
        }
        n.deliver = nd;
        std::set<std::string> my_s = on_s;
        DeliverSet ns;
        for (auto& i : n.stream) {
          if (!my_s.count(i.as_str)) {
            my_s.insert(i.as_str);
            ns.insert(i);
          } else if (i.must_deliver) {
            ns.insert(i);
          }
        }
        n.stream = ns;
        Actions my_a = on_a;
        if (!n.actions.drop()) {
          n.actions.clear_intersection(my_a);
          my_a.push(n.actions);
        }
        for (auto& c : n.children) f(c, my_a, my_d, my_s);
        std::vector<PNode> kept;
        for (auto& c : n.children)
          if (!c.actions.drop() || !c.children.empty() || !c.deliver.empty()) kept.push_back(std::move(c));
        n.children = std::move(kept);
      };
  f(root, Actions(), {}, {});
}

// 641-687
void PTree::prune_packet_conditions() {
  if (layer == FilterLayer::PacketContinue) return;
  std::function<void(PNode&, bool)> f = [&](PNode& n, bool can_prune) {
    if (!n.pred.on_packet()) return;
    bool next = windows_all_excl(n.children);
    for (auto& c : n.children) f(c, next);
    if (!can_prune) return;
    while (n.children.size() == 1 && n.children[0].pred.on_packet()) {
      PNode& c = n.children[0];
      if (extracts_protocol(c, layer)) break;
      n.actions.push(c.actions);
      n.deliver.insert(c.deliver.begin(), c.deliver.end());
      n.stream.insert(c.stream.begin(), c.stream.end());
      std::vector<PNode> gc = std::move(c.children);
      n.children = std::move(gc);
    }
  };
  f(root, windows_all_excl(root.children));
}

// 693-748
void PTree::prune_redundant_branches() {
  if (layer == FilterLayer::PacketContinue) return;
  std::function<void(PNode&, bool)> f = [&](PNode& n, bool can_prune) {
    if (!is_prev_layer_pred(n.pred, layer)) return;
    bool next = windows_all_excl(n.children);
    for (auto& c : n.children) f(c, next);
    if (!can_prune) return;
    std::vector<PNode> must_keep, could_drop;
    for (auto& c : n.children) {
      bool keep = !c.actions.drop() || !c.stream.empty() || !c.deliver.empty() || !is_prev_layer_pred(c.pred, layer) ||
                  extracts_protocol(c, layer);
      (keep ? must_keep : could_drop).push_back(c);
    }
    std::vector<PNode> nc;
    for (auto& c : could_drop) {
      bool all = true;
      for (auto& o : n.children) all = all && all_paths_eq(c, o);
      if (all) {
        for (auto& g : c.children) nc.push_back(g);
      } else {
        nc.push_back(c);
      }
    }
    for (auto& c : must_keep) nc.push_back(c);
    rust_stable_sort(nc);
    std::vector<PNode> dd;
    for (auto& c : nc)
      if (dd.empty() || !dd.back().same_contents(c)) dd.push_back(std::move(c));
    n.children = std::move(dd);
  };
  f(root, windows_all_excl(root.children));
}

// 752-776
void PTree::collapse() {
  if (layer == FilterLayer::PacketDeliver || layer == FilterLayer::ConnectionDeliver) {
    collapsed = true;
    Deliver d;
    if (get_single_callback(d)) {
      clear();
      root.deliver.insert(d);
      update_size();
      return;
    }
  }
  prune_redundant_branches();
  prune_packet_conditions();
  prune_branches();
  sort();
  mark_mutual_exclusion();
  update_size();
}

std::string PTree::pprint() const {
  std::string s;
  std::function<void(const PNode&, const std::string&, bool)> f = [&](const PNode& n, const std::string& prefix,
                                                                       bool last) {
    s += prefix + (last ? "`- " : "|- ") + std::to_string(n.id) + ": " + n.display() + "\n";
    std::string p2 = prefix + (last ? "   " : "|  ");
    for (size_t k = 0; k < n.children.size(); ++k) f(n.children[k], p2, k + 1 == n.children.size());
  };
  f(root, "", true);
  return std::string("Tree ") + filter_layer_str(layer) + "\n," + s;
}

std::string PTree::to_filter_string() const {
  if (root.children.empty()) return "";
  std::vector<std::string> all;
  std::function<void(const PNode&, std::string)> f = [&](const PNode& p, std::string curr) {
    if (curr.empty()) curr.push_back('(');
    else curr += "(" + p.pred.str() + ")";
    if (p.children.empty()) {
      all.push_back(curr + ")");
    } else {
      if (curr != "(") curr += " and ";
      for (auto& c : p.children) f(c, curr);
    }
  };
  f(root, "");
  std::string s;
  for (size_t k = 0; k < all.size(); ++k) {
    if (k) s += " or ";
    s += all[k];
  }
  return s;
}

// filtergen/src/lib.rs:241-261
PTree filter_subtree(FilterLayer layer, const std::vector<SubscriptionSpec>& subs) {
  PTree t(layer);
  for (size_t id = 0; id < subs.size(); ++id) {
    const auto& spec = subs[id];
    Filter f = Filter::make(spec.filter);
    Deliver d;
    d.id = id;
    d.as_str = spec.as_str();
    d.must_deliver = spec.has_datatype("FilterStr");
    t.add_filter(f.get_patterns_flat(), spec, d);
  }
  t.collapse();
  return t;
}

}  // namespace rtn
