// Filter compiler front half: patterns, subscriptions, predicate trees.
//
// Reference map (stanford-esrg/retina):
//   core/src/filter/parser.rs:94-357     parse_filter -> Vec<RawPattern>
//   core/src/filter/pattern.rs:17-256    FlatPattern / LayeredPattern / to_fully_qualified
//   core/src/filter/ptree_flat.rs:80-267 FlatPTree (validation + prune_branches)
//   core/src/filter/mod.rs:112-152       Filter::new / get_patterns_flat
//   core/src/filter/actions.rs:17-76     ActionData bit positions (bitmask-enum, declaration order)
//   core/src/filter/datatypes.rs         DataType / Level / SubscriptionSpec action tables
//   datatypes/src/typedefs.rs:15-86      DATATYPES
//   core/src/filter/ptree.rs:10-928      FilterLayer / PNode / PTree build + collapse
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "ast.hpp"

namespace rtn {

using RawPattern = std::vector<Predicate>;
std::vector<RawPattern> parse_filter_raw(const std::string& filter);

struct FlatPattern {
  std::vector<Predicate> predicates;
  bool operator<(const FlatPattern& o) const { return predicates < o.predicates; }
  bool operator==(const FlatPattern& o) const { return predicates == o.predicates; }
  std::string str() const;
};

// LinkedHashMap<ProtocolName, Vec<Predicate>> (insertion ordered)
struct LayeredPattern {
  std::vector<std::pair<std::string, std::vector<Predicate>>> layers;
  bool add_protocol(const std::string& proto, const std::vector<Predicate>& preds);
  FlatPattern to_flat() const;
};

std::vector<LayeredPattern> to_fully_qualified(const FlatPattern& p);
// FlatPTree::new(patterns) + prune_branches + to_flat_patterns (ptree_flat.rs:91-174, 257-267)
std::vector<FlatPattern> flat_ptree_pruned(const std::vector<FlatPattern>& patterns);

// Filter::new (core/src/filter/mod.rs:113-139)
struct Filter {
  std::vector<LayeredPattern> patterns;
  static Filter make(const std::string& filter_raw);
  std::vector<FlatPattern> get_patterns_flat() const;
};

// ---------------------------------------------------------------------------------------------
// Actions (actions.rs)
namespace action {
enum : uint32_t {
  PacketContinue = 1u << 0,
  PacketDeliver = 1u << 1,
  PacketCache = 1u << 2,
  PacketTrack = 1u << 3,
  ProtoProbe = 1u << 4,
  ProtoFilter = 1u << 5,
  SessionFilter = 1u << 6,
  SessionDeliver = 1u << 7,
  SessionTrack = 1u << 8,
  UpdatePDU = 1u << 9,
  Reassemble = 1u << 10,
  ConnDeliver = 1u << 11,
  Stream = 1u << 12,
};
}

struct Actions {
  uint32_t data = 0, terminal = 0;
  void push(const Actions& a) { data |= a.data; terminal |= a.terminal; }
  bool drop() const { return data == 0 && terminal == 0; }
  void clear_intersection(const Actions& a) { data &= ~a.data; terminal &= ~a.data; }
  bool operator==(const Actions& o) const { return data == o.data && terminal == o.terminal; }
  bool operator!=(const Actions& o) const { return !(*this == o); }
  std::string debug() const;
};

// ---------------------------------------------------------------------------------------------
// Datatypes / subscriptions (datatypes.rs)
enum class Level { Packet, Connection, Session, Static, Streaming };
enum class FilterLayer { PacketContinue, Packet, Protocol, Session, ConnectionDeliver, PacketDeliver };
const char* filter_layer_str(FilterLayer l);

struct DataType {
  Level level = Level::Static;
  bool needs_parse = false, track_sessions = false, needs_update = false, needs_reassembly = false,
       needs_packet_track = false;
  std::string as_str;
  static DataType connection(const std::string& n);
  static DataType session(const std::string& n);
  static DataType packet(const std::string& n);
  static DataType static_(const std::string& n);
  static DataType pktlist(const std::string& n, bool reassembly);
  bool should_deliver(FilterLayer l, const Predicate& p, Level sub_level) const;
  bool can_deliver(FilterLayer l, const Predicate& p) const;
};

// DATATYPES (datatypes/src/typedefs.rs:15-86). Returns false if unknown.
bool lookup_datatype(const std::string& name, DataType& out);

struct MatchingActions {
  Actions if_matched, if_matching;
};

struct SubscriptionSpec {
  std::vector<DataType> datatypes;
  std::string filter;
  std::string callback;
  Level level = Level::Static;

  SubscriptionSpec() = default;
  SubscriptionSpec(std::string f, std::string cb) : filter(std::move(f)), callback(std::move(cb)) {}
  void add_datatype(const DataType& d);
  void validate_spec() const;  // throws FilterError
  std::string as_str() const;
  bool has_datatype(const std::string& n) const;
  bool should_deliver(FilterLayer l, const Predicate& p) const;
  bool deliver_on_session() const;
  bool should_stream(FilterLayer l, const Predicate& p) const;
  bool pred_is_prev_layer(const Predicate& p, FilterLayer l) const;  // Predicate::is_prev_layer
  MatchingActions packet_continue() const;
  MatchingActions packet_filter() const;
  MatchingActions proto_filter() const;
  MatchingActions session_filter() const;
  Actions with_term_filter(FilterLayer l, const Predicate& p) const;
  Actions with_nonterm_filter(FilterLayer l) const;

  static SubscriptionSpec default_connection();
  static SubscriptionSpec default_session();
  static SubscriptionSpec default_packet();
  static SubscriptionSpec default_streaming();
};

// ---------------------------------------------------------------------------------------------
// PTree (ptree.rs)
struct Deliver {
  size_t id = 0;
  std::string as_str;
  bool must_deliver = false;
  bool operator==(const Deliver& o) const { return id == o.id && as_str == o.as_str && must_deliver == o.must_deliver; }
  bool operator<(const Deliver& o) const {
    if (id != o.id) return id < o.id;
    if (as_str != o.as_str) return as_str < o.as_str;
    return must_deliver < o.must_deliver;
  }
};
// HashSet<Deliver> in the reference; kept ordered by id here so every walk is deterministic.
using DeliverSet = std::set<Deliver>;

struct PNode {
  size_t id = 0;
  Predicate pred;
  Actions actions;
  DeliverSet deliver;
  DeliverSet stream;
  std::vector<size_t> patterns;
  std::vector<PNode> children;
  bool if_else = false;

  std::string display() const;
  bool same_contents(const PNode& o) const {  // PartialEq for PNode (ptree.rs:871-876)
    return pred == o.pred && actions == o.actions && deliver == o.deliver;
  }
};

struct PTree {
  PNode root;
  size_t size = 1;
  Actions actions;
  FilterLayer layer = FilterLayer::PacketContinue;
  bool collapsed = false;

  explicit PTree(FilterLayer l);
  void add_filter(const std::vector<FlatPattern>& patterns, const SubscriptionSpec& sub, const Deliver& d);
  void collapse();
  void prune_branches();
  void update_size();
  void clear();
  const PNode* get_subtree(size_t id) const;
  std::string pprint() const;  // "Tree <layer>\n,<tree>" like Display for PTree
  std::string to_filter_string() const;

 private:
  void build_tree(const std::vector<FlatPattern>& patterns, const SubscriptionSpec& sub, const Deliver& d);
  void add_pattern(const FlatPattern& pattern, size_t pattern_id, const SubscriptionSpec& sub, const Deliver& d);
  void sort();
  void mark_mutual_exclusion();
  void prune_packet_conditions();
  void prune_redundant_branches();
  bool get_single_callback(Deliver& out) const;
};

// filter_subtree (filtergen/src/lib.rs:241-261): every subscription's patterns into one tree.
PTree filter_subtree(FilterLayer layer, const std::vector<SubscriptionSpec>& subs);

// Subscription spec file (the #[subscription("spec.toml")] format, filtergen/src/parse.rs:7-66).
std::vector<SubscriptionSpec> parse_subscription_toml(const std::string& text);

}  // namespace rtn
