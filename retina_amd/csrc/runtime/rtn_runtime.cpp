// C-ABI runtime: compile subscription specs, build the specialised gfx950 kernel with hiprtc,
// load it and launch it. See include/retina_pc.h for the contract and reference map.
#include "retina_pc.h"
#include "retina_ct.h"
#include "retina_hw.h"
#include "retina_pd.h"

#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../filtergen/codegen.hpp"
#include "rtn_error.hpp"

namespace {
thread_local std::string g_err;
}  // namespace

int32_t rtn::set_error(int32_t code, const std::string& msg) {
  g_err = msg;
  return code;
}

namespace {

#include "pc_kernel_src.inc"  // kPcKernelSrc: csrc/kernels/pc_kernel.hip as a string literal
#include "ct_kernel_src.inc"  // kCtKernelSrc: csrc/kernels/ct_kernel.hip

int32_t fail(int32_t code, const std::string& msg) { return rtn::set_error(code, msg); }

size_t copy_text(const std::string& s, char* buf, size_t cap) {
  if (buf && cap > 0) {
    size_t n = s.size() < cap - 1 ? s.size() : cap - 1;
    memcpy(buf, s.data(), n);
    buf[n] = 0;
  }
  return s.size();
}

std::string env_defines();
std::string kernel_template();

std::string build_source(const rtn::PacketProgram& prog) {
  const std::string tpl = kernel_template();
  const std::string marker = "//@@RTN_FILTER@@";
  size_t at = tpl.find(marker);
  std::string head = "#define RTN_DELIVER_WORDS " + std::to_string(prog.deliver_words()) + "\n" +
                     "#define RTN_CONN_WORDS " + std::to_string(prog.conn_deliver_words()) + "\n" +
                     "#define RTN_PD_STMTS " + std::to_string(prog.pd_stmts.size()) + "\n" +
                     "#define RTN_PD_FACTS " + std::to_string(prog.pd_facts.size()) + "\n" + env_defines();
  const std::string& body = head.find("RTN_BRANCHY_FILTER") != std::string::npos ? prog.hip_body_branchy
                            : head.find("RTN_CHAIN_FILTER") != std::string::npos ? prog.hip_body_chain
                            : head.find("RTN_FOLD_ACT") != std::string::npos     ? prog.hip_body_fold
                                                                                  : prog.hip_body;
  std::string src = head + tpl.substr(0, at) + body + tpl.substr(at + marker.size());
  const std::string cmarker = "//@@RTN_CONN_FILTER@@";
  size_t cat = src.find(cmarker);
  src = src.substr(0, cat) + prog.hip_conn_body + src.substr(cat + cmarker.size());
  const std::string dmarker = "//@@RTN_PD_FILTER@@";
  size_t dat = src.find(dmarker);
  return src.substr(0, dat) + prog.hip_pd_body + src.substr(dat + dmarker.size());
}

// Kernel experiments: only a library built with -DRTN_EXPERIMENTS (tools/build_experiments.py)
// reads RTN_KERNEL_DEFINES="A,B=1" (prepended #defines) and RTN_KERNEL_TEMPLATE=<file> (a
// variant of pc_kernel.hip). The product library has neither, so no environment variable can
// change what a kernel computes or where it writes.
std::string kernel_template() {
#ifdef RTN_EXPERIMENTS
  if (const char* f = getenv("RTN_KERNEL_TEMPLATE")) {
    std::ifstream in(f);
    std::stringstream ss;
    ss << in.rdbuf();
    if (in && !ss.str().empty()) return ss.str();
  }
#endif
  return kPcKernelSrc;
}

// The connection-lookup kernel source: the embedded ct_kernel.hip, or (experiments build only)
// RTN_CT_TEMPLATE=<file>, so that tools/ct_ab.py can time two variants in one process.
std::string ct_template() {
#ifdef RTN_EXPERIMENTS
  if (const char* f = getenv("RTN_CT_TEMPLATE")) {
    std::ifstream in(f);
    std::stringstream ss;
    ss << in.rdbuf();
    if (in && !ss.str().empty()) return ss.str();
  }
#endif
  return kCtKernelSrc;
}

std::string env_defines() {
  std::string head;
#ifdef RTN_EXPERIMENTS
  if (const char* d = getenv("RTN_KERNEL_DEFINES")) {
    std::string all = d, tok;
    for (size_t k = 0; k <= all.size(); ++k) {
      if (k == all.size() || all[k] == ',') {
        if (!tok.empty()) head += "#define " + tok + "\n";
        tok.clear();
      } else if (all[k] != ' ') {
        tok += all[k] == '=' ? ' ' : all[k];
      }
    }
  }
#endif
  return head;
}

std::string json_str(const std::string& s) {
  std::string o = "\"";
  for (char c : s) {
    if (c == '"' || c == '\\') o += '\\';
    o += c;
  }
  return o + "\"";
}

std::string node_json(const rtn::PNode& n) {
  std::string o = "{\"id\":" + std::to_string(n.id) + ",\"pred\":" + json_str(n.pred.str()) +
                  ",\"unary\":" + (n.pred.is_unary() ? "true" : "false") + ",\"protocol\":" + json_str(n.pred.protocol) +
                  ",\"data\":" + std::to_string(n.actions.data) + ",\"terminal\":" + std::to_string(n.actions.terminal) +
                  ",\"if_else\":" + (n.if_else ? "true" : "false") + ",\"deliver\":[";
  bool first = true;
  for (auto& d : n.deliver) {
    o += (first ? "" : ",") + std::to_string(d.id);
    first = false;
  }
  o += "],\"stream\":[";
  first = true;
  for (auto& d : n.stream) {
    o += (first ? "" : ",") + std::to_string(d.id);
    first = false;
  }
  o += "],\"children\":[";
  for (size_t k = 0; k < n.children.size(); ++k) o += (k ? "," : "") + node_json(n.children[k]);
  return o + "]}";
}

// The PacketDeliver program for the host: its facts (what the host computes per connection) and
// its statements in code order, each with the session loops around it.
std::string pd_json(const rtn::PacketProgram& prog) {
  std::string o = "{\"facts\":[";
  for (size_t k = 0; k < prog.pd_facts.size(); ++k) {
    const auto& f = prog.pd_facts[k];
    o += std::string(k ? "," : "") + "{\"kind\":" + (f.kind == rtn::PdFact::Service ? "\"service\"" : "\"session\"") +
         ",\"pred\":" + json_str(f.pred) + ",\"protocol\":" + json_str(f.protocol) + "}";
  }
  o += "],\"stmts\":[";
  for (size_t k = 0; k < prog.pd_stmts.size(); ++k) {
    const auto& st = prog.pd_stmts[k];
    o += std::string(k ? "," : "") + "{\"sub\":" + std::to_string(st.d.sub_id) +
         ",\"payload\":" + (st.d.payload ? "true" : "false") + ",\"callback\":" + json_str(st.d.callback) + ",\"loops\":[";
    for (size_t j = 0; j < st.loops.size(); ++j)
      o += std::string(j ? "," : "") + "[" + std::to_string(st.loops[j].first) + "," + std::to_string(st.loops[j].second) + "]";
    o += "]}";
  }
  return o + "]}";
}

uint64_t fnv1a(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
  return h;
}

std::mutex g_cache_mu;
std::map<uint64_t, std::shared_ptr<std::vector<uint8_t>>> g_cache;  // source hash -> code object

// Extra hiprtc options, experiments build only: RTN_KERNEL_OPTS="-mllvm -x ..." (space-separated),
// so tools/ab.py can time compiler settings against each other in one process.
std::vector<std::string> env_opts() {
  std::vector<std::string> o;
#ifdef RTN_EXPERIMENTS
  if (const char* e = getenv("RTN_KERNEL_OPTS")) {
    std::stringstream ss(e);
    std::string t;
    while (ss >> t) o.push_back(t);
  }
#endif
  return o;
}

int32_t compile_code_object(const std::string& src, std::shared_ptr<std::vector<uint8_t>>& out) {
  const std::vector<std::string> extra = env_opts();
  std::string key = src;
  for (const auto& e : extra) key += "\n//opt " + e;
  const uint64_t h = fnv1a(key);
  {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    auto it = g_cache.find(h);
    if (it != g_cache.end()) {
      out = it->second;
      return RTN_OK;
    }
  }
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "rtn_pc_kernel.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
    return fail(RTN_ECOMPILE, "hiprtcCreateProgram failed");
  std::string arch = "--offload-arch=gfx950";
  if (const char* a = getenv("RTN_OFFLOAD_ARCH")) arch = std::string("--offload-arch=") + a;
  std::vector<const char*> opts = {arch.c_str(), "-O3", "-std=c++17"};
  for (const auto& e : extra) opts.push_back(e.c_str());
  hiprtcResult r = hiprtcCompileProgram(prog, (int)opts.size(), opts.data());
  size_t ls = 0;
  hiprtcGetProgramLogSize(prog, &ls);
  std::string log(ls, '\0');
  if (ls) hiprtcGetProgramLog(prog, &log[0]);
  if (r != HIPRTC_SUCCESS) {
    hiprtcDestroyProgram(&prog);
    return fail(RTN_ECOMPILE, std::string("hiprtc: ") + hiprtcGetErrorString(r) + "\n" + log);
  }
  size_t cs = 0;
  hiprtcGetCodeSize(prog, &cs);
  auto code = std::make_shared<std::vector<uint8_t>>(cs);
  hiprtcGetCode(prog, reinterpret_cast<char*>(code->data()));
  hiprtcDestroyProgram(&prog);
  {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    g_cache[h] = code;
  }
  out = code;
  return RTN_OK;
}

}  // namespace

int32_t rtn::compile_hip(const std::string& src, std::shared_ptr<std::vector<uint8_t>>& out) {
  return compile_code_object(src, out);
}

namespace {

// kernel argument block; must match struct rtn_args in pc_kernel.hip
struct KArgs {
  const unsigned char* slab;
  uint64_t stride;
  const unsigned short* dlen;
  uint32_t n;
  uint32_t flags;
  uint64_t* pc_bm;
  uint64_t* fwd_bm;
  rtn_l4ctx_t* recs;
  unsigned char* addr6;
  uint64_t* dlv_bm;
  uint64_t* dlv_recs;
  uint32_t* counters;
  const unsigned char* ext;
  rtn_conn_t* conn;
  uint64_t* conn_dlv;
  const uint32_t* ext_chunk;
  uint32_t ext_rows;
  uint32_t cpw;
  uint64_t* seqack;
};

// Groups per wave of a kernel (RTN_PD_GPW / RTN_CT_GPW): the default, unless an RTN_KERNEL_DEFINES
// experiment (experiments build only) overrides it (the launch's block size follows it).
uint32_t groups_per_wave(const char* name, uint32_t dflt) {
  const std::string d = env_defines(), key = std::string("#define ") + name + " ";
  size_t at = d.find(key);
  if (at == std::string::npos) return dflt;
  uint32_t g = (uint32_t)strtoul(d.c_str() + at + key.size(), nullptr, 10);
  return (g == 1u || g == 2u || g == 4u || g == 8u) ? g : dflt;
}
uint32_t pd_groups_per_wave() { return groups_per_wave("RTN_PD_GPW", 1u); }

// must match struct rtn_pd_args in pc_kernel.hip
struct PdArgs {
  const uint64_t* fwd_bm;
  const rtn_l4ctx_t* recs;
  const uint8_t* addr6;
  const rtn_conn_t* conn;
  const rtn_ct_entry_t* ct;
  const uint16_t* dlen;
  const uint32_t* state;
  uint32_t state_slots;
  uint32_t n;
  uint32_t* counts;
  uint64_t* pd_bm;
};

// must match struct rtn_idx_args in pc_kernel.hip
struct IdxArgs {
  const uint64_t* bm;
  uint32_t n;
  uint32_t nblocks;
  uint32_t* block_sum;
  uint32_t* idx;
  uint32_t* n_set;
  uint32_t* chunk_base;
};
constexpr uint32_t RTN_IDX_WORDS = 4096;  // bitmap words per block, must match pc_kernel.hip

// Waves per SIMD a kernel reaches in blocks of `threads` (the runtime's occupancy calculator:
// registers and LDS); 0 if it cannot say.
uint32_t waves_per_simd(hipFunction_t f, uint32_t threads) {
  int blocks = 0;
  if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, f, (int)threads, 0) != hipSuccess || blocks <= 0) {
    (void)hipGetLastError();
    return 0;
  }
  return (uint32_t)blocks * (threads / 64u) / 4u;  // 4 SIMDs per CU
}

}  // namespace

struct rtn_program {
  rtn::PacketProgram prog;
  std::string source;
  std::shared_ptr<std::vector<uint8_t>> code;
};

struct rtn_pc {
  rtn_program* owned = nullptr;  // set when created from a spec
  const rtn_program* program = nullptr;
  int device = 0;
  hipModule_t module = nullptr;
  hipFunction_t fn = nullptr;        // rtn_pc_kernel: monolithic slots, any stride (multiple of 64)
  hipFunction_t fn_s64 = nullptr;    // rtn_pc_kernel_s64: 64-byte slots
  hipFunction_t fn_split = nullptr;  // rtn_pc_kernel_split: 64-byte slots + ext
  hipFunction_t fn_splitc = nullptr; // rtn_pc_kernel_splitc: 64-byte slots + compact ext rows
  hipFunction_t fn_conn[4] = {};     // the same four with the connection stage (*_conn), same order
  hipFunction_t fn_pd = nullptr;     // rtn_pd_kernel: the PacketDeliver filter (rtn_pd_run)
  hipFunction_t fn_idx[3] = {};      // rtn_idx_count / rtn_idx_scan / rtn_idx_write (rtn_pc_index)
  uint32_t* idx_block_sum = nullptr; // their per-block sums (RTN_MAX_FRAMES / 64 / RTN_IDX_WORDS)
  uint32_t blocks = 0;
  uint32_t threads = 256;  // threads per block of the packet kernel (4 waves, one chunk each)
  uint32_t splitc_cpw = 1;  // chunks per wave of rtn_pc_kernel_splitc (rtn_args.cpw)
  uint32_t splitc_cpw_conn = 1;  // ... of rtn_pc_kernel_splitc_conn
  // used when the caller passes no counters: word RTN_CNT_STATUS accumulates the status bits of
  // such runs until rtn_pc_take_status reads and clears them (the other words are never read)
  uint32_t* scratch_counters = nullptr;
  hipEvent_t last_nc = nullptr;  // recorded after each run without counters (rtn_pc_take_status)
  hipStream_t own = nullptr;     // private non-blocking stream of rtn_pc_take_status
  ~rtn_pc() {
    if (last_nc) (void)hipEventDestroy(last_nc);
    if (own) (void)hipStreamDestroy(own);
    if (scratch_counters) (void)hipFree(scratch_counters);
    if (idx_block_sum) (void)hipFree(idx_block_sum);
    if (module) (void)hipModuleUnload(module);
    delete owned;
  }
};

extern "C" {

const char* rtn_last_error(void) { return g_err.c_str(); }

int32_t rtn_program_compile(const char* spec, size_t len, rtn_program_t** out) {
  if (!spec || !out) return fail(RTN_EINVAL, "null argument");
  try {
    auto subs = rtn::parse_subscription_toml(std::string(spec, len));
    auto p = std::make_unique<rtn_program>();
    p->prog = rtn::compile_packet_program(subs);
    p->source = build_source(p->prog);
    *out = p.release();
    return RTN_OK;
  } catch (const rtn::FilterError& e) {
    return fail(RTN_EFILTER, e.what());
  } catch (const std::exception& e) {
    return fail(RTN_EFILTER, std::string("internal error: ") + e.what());
  }
}

int32_t rtn_program_compile_filter(const char* filter, const char* datatypes, const char* callback,
                                   rtn_program_t** out) {
  if (!filter || !datatypes || !out) return fail(RTN_EINVAL, "null argument");
  try {
    rtn::SubscriptionSpec s(filter, callback ? callback : "cb");
    std::string dts = datatypes, tok;
    auto flush = [&]() {
      size_t b = tok.find_first_not_of(" \t"), e = tok.find_last_not_of(" \t");
      if (b != std::string::npos) {
        std::string t = tok.substr(b, e - b + 1);
        rtn::DataType dt;
        if (!rtn::lookup_datatype(t, dt)) throw rtn::FilterError("Invalid datatype: " + t);
        s.add_datatype(dt);
      }
      tok.clear();
    };
    for (char c : dts) {
      if (c == ',') flush();
      else tok.push_back(c);
    }
    flush();
    if (s.datatypes.empty()) throw rtn::FilterError("subscription without datatypes");
    auto p = std::make_unique<rtn_program>();
    p->prog = rtn::compile_packet_program({s});
    p->source = build_source(p->prog);
    *out = p.release();
    return RTN_OK;
  } catch (const rtn::FilterError& e) {
    return fail(RTN_EFILTER, e.what());
  } catch (const std::exception& e) {
    return fail(RTN_EFILTER, std::string("internal error: ") + e.what());
  }
}

int32_t rtn_program_info(const rtn_program_t* p, rtn_program_info_t* info) {
  if (!p || !info) return fail(RTN_EINVAL, "null argument");
  info->n_subscriptions = (uint32_t)p->prog.subs.size();
  info->n_deliver_stmts = (uint32_t)p->prog.delivers.size();
  info->deliver_words = p->prog.deliver_words();
  info->tree_size = (uint32_t)p->prog.tree.size;
  info->n_conn_stmts = (uint32_t)p->prog.conn_delivers.size();
  info->conn_words = p->prog.conn_deliver_words();
  info->conn_tree_size = (uint32_t)p->prog.conn_tree.size;
  info->n_pd_stmts = (uint32_t)p->prog.pd_stmts.size();
  info->n_pd_facts = (uint32_t)p->prog.pd_facts.size();
  info->pd_tree_size = (uint32_t)p->prog.pd_tree.size;
  return RTN_OK;
}

size_t rtn_program_hw_filter(const rtn_program_t* p, char* buf, size_t cap) {
  return p ? copy_text(p->prog.hw_filter, buf, cap) : 0;
}
int32_t rtn_program_hw_rules(const rtn_program_t* p, rtn_flow_validate_fn validate, void* user,
                             rtn_flow_rule_t* rules, uint32_t cap, uint32_t* n_rules) {
  if (!p) return fail(RTN_EINVAL, "null program");
  return rtn_hw_rules(p->prog.hw_filter.c_str(), validate, user, rules, cap, n_rules);
}
size_t rtn_program_conn_tree(const rtn_program_t* p, char* buf, size_t cap) {
  return p ? copy_text(p->prog.conn_tree.pprint(), buf, cap) : 0;
}
size_t rtn_program_conn_rust(const rtn_program_t* p, char* buf, size_t cap) {
  return p ? copy_text(p->prog.rust_conn_listing, buf, cap) : 0;
}
size_t rtn_program_tree_json(const rtn_program_t* p, uint32_t layer, char* buf, size_t cap) {
  if (!p || layer > 2) return 0;
  const rtn::PNode& r = layer == 0 ? p->prog.tree.root : layer == 1 ? p->prog.conn_tree.root : p->prog.pd_tree.root;
  return copy_text(node_json(r), buf, cap);
}
size_t rtn_program_pd_json(const rtn_program_t* p, char* buf, size_t cap) {
  return p ? copy_text(pd_json(p->prog), buf, cap) : 0;
}
size_t rtn_program_pd_rust(const rtn_program_t* p, char* buf, size_t cap) {
  return p ? copy_text(p->prog.rust_pd_listing, buf, cap) : 0;
}

// The callback order of one frame from its counts: statements of one session-loop body repeat as
// a block, facts[fact] times (deliver_filter.rs:123-151); a statement fires in a pass iff its
// count is non-zero. Recursion over the loop nesting of consecutive statements.
static size_t pd_replay_rec(const std::vector<rtn::PdStmt>& st, const uint32_t* counts, const uint32_t* facts,
                            size_t b, size_t e, size_t depth, uint32_t* out, size_t cap, size_t n) {
  size_t i = b;
  while (i < e) {
    if (st[i].loops.size() == depth) {
      if (counts[i]) {
        if (n < cap && out) out[n] = (uint32_t)i;
        ++n;
      }
      ++i;
      continue;
    }
    const uint32_t node = st[i].loops[depth].first, fact = st[i].loops[depth].second;
    size_t j = i;
    while (j < e && st[j].loops.size() > depth && st[j].loops[depth].first == node) ++j;
    for (uint32_t r = 0; r < facts[fact]; ++r) n = pd_replay_rec(st, counts, facts, i, j, depth + 1, out, cap, n);
    i = j;
  }
  return n;
}

int32_t rtn_program_pd_replay(const rtn_program_t* p, const uint32_t* counts, const uint32_t* facts, uint32_t* out,
                              uint32_t cap, uint32_t* n) {
  if (!p || !counts || !n || (!facts && !p->prog.pd_facts.empty())) return fail(RTN_EINVAL, "null argument");
  const size_t k = pd_replay_rec(p->prog.pd_stmts, counts, facts, 0, p->prog.pd_stmts.size(), 0, out, cap, 0);
  *n = (uint32_t)k;
  if (k > cap) return fail(RTN_ERANGE, "replay longer than the output capacity (*n holds the length)");
  return RTN_OK;
}

int32_t rtn_program_conn_table(const rtn_program_t* p, uint32_t* sub_ids, uint8_t* kinds, uint32_t cap) {
  if (!p) return fail(RTN_EINVAL, "null program");
  const auto& d = p->prog.conn_delivers;
  if (cap < d.size()) return fail(RTN_ERANGE, "statement table capacity too small");
  for (size_t k = 0; k < d.size(); ++k) {
    if (sub_ids) sub_ids[k] = d[k].sub_id;
    if (kinds) kinds[k] = (uint8_t)d[k].kind;
  }
  return RTN_OK;
}

size_t rtn_program_tree(const rtn_program_t* p, char* buf, size_t cap) {
  return p ? copy_text(p->prog.tree.pprint(), buf, cap) : 0;
}
size_t rtn_program_rust(const rtn_program_t* p, char* buf, size_t cap) {
  return p ? copy_text(p->prog.rust_listing, buf, cap) : 0;
}
size_t rtn_program_source(const rtn_program_t* p, char* buf, size_t cap) {
  return p ? copy_text(p->source, buf, cap) : 0;
}

int32_t rtn_program_deliver_table(const rtn_program_t* p, uint32_t* sub_ids, uint8_t* is_payload, uint32_t cap) {
  if (!p) return fail(RTN_EINVAL, "null program");
  const auto& d = p->prog.delivers;
  if (cap < d.size()) return fail(RTN_ERANGE, "deliver table capacity too small");
  for (size_t k = 0; k < d.size(); ++k) {
    if (sub_ids) sub_ids[k] = d[k].sub_id;
    if (is_payload) is_payload[k] = d[k].payload ? 1 : 0;
  }
  return RTN_OK;
}

size_t rtn_program_deliver_callback(const rtn_program_t* p, uint32_t k, char* buf, size_t cap) {
  if (!p || k >= p->prog.delivers.size()) return 0;
  return copy_text(p->prog.delivers[k].callback, buf, cap);
}

int32_t rtn_program_code_object(rtn_program_t* p, const uint8_t** data, size_t* len) {
  if (!p || !data || !len) return fail(RTN_EINVAL, "null argument");
  if (!p->code) {
    int32_t rc = compile_code_object(p->source, p->code);
    if (rc) return rc;
  }
  *data = p->code->data();
  *len = p->code->size();
  return RTN_OK;
}

void rtn_program_destroy(rtn_program_t* p) { delete p; }

int32_t rtn_pc_create_from_program(rtn_program_t* p, int device, rtn_pc_t** out) {
  if (!p || !out) return fail(RTN_EINVAL, "null argument");
  const uint8_t* code;
  size_t len;
  int32_t rc = rtn_program_code_object(p, &code, &len);
  if (rc) return rc;
  auto pc = std::make_unique<rtn_pc>();
  pc->program = p;
  pc->device = device;
  if (hipSetDevice(device) != hipSuccess) return fail(RTN_EDEVICE, "hipSetDevice failed");
  hipError_t e = hipModuleLoadData(&pc->module, code);
  if (e != hipSuccess) return fail(RTN_EDEVICE, std::string("hipModuleLoadData: ") + hipGetErrorString(e));
  e = hipModuleGetFunction(&pc->fn, pc->module, "rtn_pc_kernel");
  if (e != hipSuccess) return fail(RTN_EDEVICE, std::string("hipModuleGetFunction: ") + hipGetErrorString(e));
  e = hipModuleGetFunction(&pc->fn_s64, pc->module, "rtn_pc_kernel_s64");
  if (e != hipSuccess) return fail(RTN_EDEVICE, std::string("hipModuleGetFunction: ") + hipGetErrorString(e));
  e = hipModuleGetFunction(&pc->fn_split, pc->module, "rtn_pc_kernel_split");
  if (e != hipSuccess) return fail(RTN_EDEVICE, std::string("hipModuleGetFunction: ") + hipGetErrorString(e));
  e = hipModuleGetFunction(&pc->fn_splitc, pc->module, "rtn_pc_kernel_splitc");
  if (e != hipSuccess) return fail(RTN_EDEVICE, std::string("hipModuleGetFunction: ") + hipGetErrorString(e));
  {
    const char* names[4] = {"rtn_pc_kernel_conn", "rtn_pc_kernel_s64_conn", "rtn_pc_kernel_split_conn",
                            "rtn_pc_kernel_splitc_conn"};
    for (int k = 0; k < 4; ++k) {
      e = hipModuleGetFunction(&pc->fn_conn[k], pc->module, names[k]);
      if (e != hipSuccess) return fail(RTN_EDEVICE, std::string("hipModuleGetFunction: ") + hipGetErrorString(e));
    }
  }
  // two consecutive chunks per wave when the compact split kernel's occupancy (registers, VGPRs
  // and AGPRs, and LDS, as the runtime computes it) is below 4 waves per SIMD: see the chunk loop
  // in pc_kernel.hip
  auto cpw_for = [pc = pc.get()](hipFunction_t f, const char* name) {
    const uint32_t waves = waves_per_simd(f, pc->threads);
    const uint32_t cpw = waves != 0 && waves < 4 ? 2u : 1u;
#ifdef RTN_EXPERIMENTS
    if (getenv("RTN_DEBUG")) fprintf(stderr, "%s: %u waves per SIMD, %u chunks per wave\n", name, waves, cpw);
#else
    (void)name;
#endif
    return cpw;
  };
  pc->splitc_cpw = cpw_for(pc->fn_splitc, "rtn_pc_kernel_splitc");
  pc->splitc_cpw_conn = cpw_for(pc->fn_conn[3], "rtn_pc_kernel_splitc_conn");
  e = hipModuleGetFunction(&pc->fn_pd, pc->module, "rtn_pd_kernel");
  if (e != hipSuccess) return fail(RTN_EDEVICE, std::string("hipModuleGetFunction: ") + hipGetErrorString(e));
  {
    const char* names[3] = {"rtn_idx_count", "rtn_idx_scan", "rtn_idx_write"};
    for (int k = 0; k < 3; ++k) {
      e = hipModuleGetFunction(&pc->fn_idx[k], pc->module, names[k]);
      if (e != hipSuccess) return fail(RTN_EDEVICE, std::string("hipModuleGetFunction: ") + hipGetErrorString(e));
    }
  }
  e = hipMalloc(&pc->idx_block_sum, (RTN_MAX_FRAMES / 64u / RTN_IDX_WORDS) * sizeof(uint32_t));
  if (e != hipSuccess) return fail(RTN_EDEVICE, std::string("hipMalloc: ") + hipGetErrorString(e));
  e = hipMalloc(&pc->scratch_counters, RTN_COUNTERS_BYTES);
  if (e != hipSuccess) return fail(RTN_EDEVICE, std::string("hipMalloc: ") + hipGetErrorString(e));
  e = hipMemset(pc->scratch_counters, 0, RTN_COUNTERS_BYTES);
  if (e != hipSuccess) return fail(RTN_EDEVICE, std::string("hipMemset: ") + hipGetErrorString(e));
  e = hipEventCreateWithFlags(&pc->last_nc, hipEventDisableTiming);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&pc->own, hipStreamNonBlocking);
  if (e != hipSuccess) return fail(RTN_EDEVICE, std::string("rtn_pc_create: ") + hipGetErrorString(e));
#ifdef RTN_EXPERIMENTS
  if (const char* g = getenv("RTN_GRID")) pc->blocks = (uint32_t)strtoul(g, nullptr, 10);
  if (const char* b = getenv("RTN_BLOCK")) pc->threads = (uint32_t)strtoul(b, nullptr, 10);
  if (const char* c = getenv("RTN_CPW")) pc->splitc_cpw = pc->splitc_cpw_conn = (uint32_t)strtoul(c, nullptr, 10);
#endif
  *out = pc.release();
  return RTN_OK;
}

int32_t rtn_pc_create(const char* spec, size_t len, int device, rtn_pc_t** out) {
  rtn_program_t* p = nullptr;
  int32_t rc = rtn_program_compile(spec, len, &p);
  if (rc) return rc;
  rc = rtn_pc_create_from_program(p, device, out);
  if (rc) {
    rtn_program_destroy(p);  // (a failed create released everything it had set up)
    return rc;
  }
  (*out)->owned = p;
  return RTN_OK;
}

int32_t rtn_pc_kernel_info(const rtn_pc_t* pc, uint32_t layout, uint32_t conn, rtn_kernel_info_t* info) {
  if (!pc || !info) return fail(RTN_EINVAL, "null argument");
  if (layout > 3) return fail(RTN_EINVAL, "layout must be 0..3");
  const hipFunction_t plain[4] = {pc->fn, pc->fn_s64, pc->fn_split, pc->fn_splitc};
  const hipFunction_t f = conn ? pc->fn_conn[layout] : plain[layout];
  int regs = 0, lds = 0;
  hipError_t e = hipFuncGetAttribute(&regs, HIP_FUNC_ATTRIBUTE_NUM_REGS, f);
  if (e == hipSuccess) e = hipFuncGetAttribute(&lds, HIP_FUNC_ATTRIBUTE_SHARED_SIZE_BYTES, f);
  if (e != hipSuccess) return fail(RTN_EDEVICE, std::string("hipFuncGetAttribute: ") + hipGetErrorString(e));
  info->regs = (uint32_t)regs;
  info->lds_bytes = (uint32_t)lds;
  info->threads = pc->threads;
  info->waves_per_simd = waves_per_simd(f, pc->threads);
  info->chunks_per_wave = layout == 3 ? (conn ? pc->splitc_cpw_conn : pc->splitc_cpw) : 1u;
  return RTN_OK;
}

int32_t rtn_pc_set_grid(rtn_pc_t* pc, uint32_t blocks) {
  if (!pc) return fail(RTN_EINVAL, "null context");
  pc->blocks = blocks;
  return RTN_OK;
}

int32_t rtn_pc_run(rtn_pc_t* pc, const rtn_batch_t* in, rtn_pc_out_t* out, void* stream) {
  if (!pc || !in || !out) return fail(RTN_EINVAL, "null argument");
  if (in->n > RTN_MAX_FRAMES) return fail(RTN_EINVAL, "batch larger than RTN_MAX_FRAMES");
  if (in->flags & ~(RTN_BATCH_DL_LE64 | RTN_BATCH_EXT_COMPACT)) return fail(RTN_EINVAL, "unknown rtn_batch_t flags");
  if ((in->flags & RTN_BATCH_EXT_COMPACT) && (!in->ext || !in->ext_chunk))
    return fail(RTN_EINVAL, "RTN_BATCH_EXT_COMPACT needs ext and ext_chunk");
  if (in->n == 0) return RTN_OK;
  if (!in->slab || !in->data_len) return fail(RTN_EINVAL, "batch slab/data_len missing");
  if (in->stride < 64 || in->stride % 64 != 0) return fail(RTN_EINVAL, "stride must be a positive multiple of 64");
  if ((reinterpret_cast<uintptr_t>(in->slab) & 15u) != 0) return fail(RTN_EINVAL, "slab must be 16-byte aligned");
  if (in->ext && in->stride != 64) return fail(RTN_EINVAL, "the split layout (ext) needs stride 64");
  if (in->ext && (reinterpret_cast<uintptr_t>(in->ext) & 15u) != 0)
    return fail(RTN_EINVAL, "ext must be 16-byte aligned");
  if (!out->pc_bitmap || !out->fwd_bitmap || !out->l4) return fail(RTN_EINVAL, "pc_bitmap/fwd_bitmap/l4 required");
  // 64-byte slots without ext: the caller must either guarantee data_len <= 64 or receive the
  // status word (RTN_STATUS_HDR_PAST_SLOT), so that a frame parsed past its slot is never silent
  if (in->stride == 64 && !in->ext && !(in->flags & RTN_BATCH_DL_LE64) && !out->counters)
    return fail(RTN_EINVAL, "64-byte slots without ext need RTN_BATCH_DL_LE64 (every data_len <= 64) or counters");
  // record arrays leave in 16-B-per-lane stores
  for (const void* o : {(const void*)out->l4, (const void*)out->addr6, (const void*)out->conn, (const void*)out->seqack})
    if ((reinterpret_cast<uintptr_t>(o) & 15u) != 0) return fail(RTN_EINVAL, "l4/addr6/conn/seqack must be 16-byte aligned");
  const uint32_t dw = pc->program->prog.deliver_words();
  if (dw > 0 && (!out->dlv_bitmap || !out->dlv_records))
    return fail(RTN_EINVAL, "program has packet-level callbacks: dlv_bitmap/dlv_records required");
  if (out->conn && pc->program->prog.conn_deliver_words() > 0 && !out->conn_dlv)
    return fail(RTN_EINVAL, "program has first-packet statements: conn_dlv required with conn");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipError_t e;
  if (out->counters) {
    e = hipMemsetAsync(out->counters, 0, RTN_COUNTERS_BYTES, s);
    if (e != hipSuccess) return fail(RTN_EDEVICE, std::string("hipMemsetAsync: ") + hipGetErrorString(e));
  }
  KArgs a;
  a.slab = in->slab;
  a.stride = in->stride;
  a.dlen = in->data_len;
  a.n = in->n;
  a.flags = (out->addr6 ? 1u : 0u) | (out->counters ? 2u : 0u) | (out->conn ? 4u : 0u) |
            ((in->flags & RTN_BATCH_DL_LE64) ? 8u : 0u) | ((in->flags & RTN_BATCH_EXT_COMPACT) ? 16u : 0u) |
            (out->seqack ? 32u : 0u);
  a.seqack = out->seqack;
  a.ext_chunk = in->ext_chunk;
  a.ext_rows = in->ext_rows;
  a.cpw = (in->ext && (in->flags & RTN_BATCH_EXT_COMPACT)) ? (out->conn ? pc->splitc_cpw_conn : pc->splitc_cpw) : 1u;
  a.pc_bm = out->pc_bitmap;
  a.fwd_bm = out->fwd_bitmap;
  a.recs = out->l4;
  a.addr6 = out->addr6;
  a.dlv_bm = out->dlv_bitmap;
  a.dlv_recs = out->dlv_records;
  a.counters = out->counters ? out->counters : pc->scratch_counters;
  a.ext = in->ext;
  a.conn = out->conn;
  a.conn_dlv = out->conn_dlv;
  const uint32_t chunks = (in->n + RTN_CHUNK_FRAMES - 1u) / RTN_CHUNK_FRAMES;
  // default: one wave per chunk (4 chunks per 256-thread block); the hardware dispatcher hands
  // out blocks as earlier ones retire, which balances the tail better than a persistent grid
  const uint32_t threads = pc->threads;
  const uint32_t per_block = (threads / 64u) * a.cpw;  // chunks per block
  const uint32_t need = (chunks + per_block - 1u) / per_block;
  uint32_t blocks = pc->blocks ? pc->blocks : need;
#ifndef RTN_EXPERIMENTS
  if (blocks > need) blocks = need;
#endif
  if (blocks == 0) blocks = 1;
  void* params[] = {&a};
  const int layout = in->ext ? ((in->flags & RTN_BATCH_EXT_COMPACT) ? 3 : 2) : (in->stride == 64 ? 1 : 0);
  const hipFunction_t plain[4] = {pc->fn, pc->fn_s64, pc->fn_split, pc->fn_splitc};
  hipFunction_t fn = out->conn ? pc->fn_conn[layout] : plain[layout];
  e = hipModuleLaunchKernel(fn, blocks, 1, 1, threads, 1, 1, 0, s, params, nullptr);
  if (e != hipSuccess) return fail(RTN_EDEVICE, std::string("hipModuleLaunchKernel: ") + hipGetErrorString(e));
  // a run without counters reports its status bits in the context's word: remember where it ends
  if (!out->counters) {
    e = hipEventRecord(pc->last_nc, s);
    if (e != hipSuccess) return fail(RTN_EDEVICE, std::string("hipEventRecord: ") + hipGetErrorString(e));
  }
  return RTN_OK;
}

int32_t rtn_pd_run(rtn_pc_t* pc, const rtn_pc_out_t* out, const rtn_ct_entry_t* ct, const uint16_t* data_len,
                   uint32_t n, const uint32_t* state, uint32_t state_slots, uint32_t* counts, uint64_t* pd_bitmap,
                   void* stream) {
  if (!pc || !out || !ct || !data_len || !pd_bitmap) return fail(RTN_EINVAL, "null argument");
  if (n > RTN_MAX_FRAMES) return fail(RTN_EINVAL, "batch larger than RTN_MAX_FRAMES");
  if (n == 0) return RTN_OK;
  if (!out->fwd_bitmap || !out->l4 || !out->addr6 || !out->conn)
    return fail(RTN_EINVAL, "fwd_bitmap, l4, addr6 and conn required");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (pc->program->prog.pd_stmts.empty()) {  // no packet-level subscription: nothing is delivered
    hipError_t e = hipMemsetAsync(pd_bitmap, 0, rtn_out_bitmap_bytes(n), s);
    return e == hipSuccess ? RTN_OK : fail(RTN_EDEVICE, std::string("hipMemsetAsync: ") + hipGetErrorString(e));
  }
  if (!state || !counts) return fail(RTN_EINVAL, "state and counts required");
  PdArgs a;
  a.fwd_bm = out->fwd_bitmap;
  a.recs = out->l4;
  a.addr6 = out->addr6;
  a.conn = out->conn;
  a.ct = ct;
  a.dlen = data_len;
  a.state = state;
  a.state_slots = state_slots;
  a.n = n;
  a.counts = counts;
  a.pd_bm = pd_bitmap;
  void* params[] = {&a};
  const uint32_t chunks = (n + RTN_CHUNK_FRAMES - 1u) / RTN_CHUNK_FRAMES;
  const uint32_t threads = RTN_CHUNK_FRAMES / pd_groups_per_wave();  // RTN_PD_THREADS in pc_kernel.hip
  hipError_t e = hipModuleLaunchKernel(pc->fn_pd, chunks, 1, 1, threads, 1, 1, 0, s, params, nullptr);
  if (e != hipSuccess) return fail(RTN_EDEVICE, std::string("hipModuleLaunchKernel: ") + hipGetErrorString(e));
  return RTN_OK;
}

int32_t rtn_pc_index(rtn_pc_t* pc, const uint64_t* bitmap, uint32_t n, uint32_t* idx, uint32_t* n_set,
                     uint32_t* chunk_base, void* stream) {
  if (!pc || !n_set || (n && (!bitmap || !idx))) return fail(RTN_EINVAL, "null argument");
  if (n > RTN_MAX_FRAMES) return fail(RTN_EINVAL, "batch larger than RTN_MAX_FRAMES");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipError_t e = hipSetDevice(pc->device);
  if (e == hipSuccess && n == 0) {
    e = hipMemsetAsync(n_set, 0, 4, s);
    if (e == hipSuccess && chunk_base) e = hipMemsetAsync(chunk_base, 0, 4, s);
    return e == hipSuccess ? RTN_OK : fail(RTN_EDEVICE, std::string("hipMemsetAsync: ") + hipGetErrorString(e));
  }
  IdxArgs a;
  a.bm = bitmap;
  a.n = n;
  a.nblocks = (uint32_t)((((uint64_t)n + 63u) / 64u + RTN_IDX_WORDS - 1u) / RTN_IDX_WORDS);
  a.block_sum = pc->idx_block_sum;
  a.idx = idx;
  a.n_set = n_set;
  a.chunk_base = chunk_base;
  void* params[] = {&a};
  const uint32_t grid[3] = {a.nblocks, 1u, a.nblocks}, threads[3] = {256u, 1024u, 256u};
  for (int k = 0; k < 3 && e == hipSuccess; ++k)
    e = hipModuleLaunchKernel(pc->fn_idx[k], grid[k], 1, 1, threads[k], 1, 1, 0, s, params, nullptr);
  return e == hipSuccess ? RTN_OK : fail(RTN_EDEVICE, std::string("rtn_pc_index: ") + hipGetErrorString(e));
}

int32_t rtn_pc_take_status(rtn_pc_t* pc, uint32_t* status) {
  if (!pc || !status) return fail(RTN_EINVAL, "null argument");
  // waits for this context's last run without counters only (not the device): the status word is
  // read and cleared on the context's own stream
  hipError_t e = hipSetDevice(pc->device);
  if (e == hipSuccess) e = hipEventSynchronize(pc->last_nc);
  if (e == hipSuccess)
    e = hipMemcpyAsync(status, pc->scratch_counters + RTN_CNT_STATUS, 4, hipMemcpyDeviceToHost, pc->own);
  if (e == hipSuccess) e = hipMemsetAsync(pc->scratch_counters + RTN_CNT_STATUS, 0, 4, pc->own);
  if (e == hipSuccess) e = hipStreamSynchronize(pc->own);
  return e == hipSuccess ? RTN_OK : fail(RTN_EDEVICE, std::string("rtn_pc_take_status: ") + hipGetErrorString(e));
}

int32_t rtn_pc_destroy(rtn_pc_t* pc) {
  delete pc;
  return RTN_OK;
}

// sizes in 64-bit arithmetic (n up to 2^32 - 1 must not wrap)
size_t rtn_out_bitmap_bytes(uint32_t n) { return (((size_t)n + 63u) / 64u) * 8u; }
static size_t chunked(uint32_t n) { return (((size_t)n + RTN_CHUNK_FRAMES - 1u) / RTN_CHUNK_FRAMES) * RTN_CHUNK_FRAMES; }
static_assert(sizeof(rtn_l4ctx_t) == 16, "rtn_l4ctx_t is 16 bytes");
size_t rtn_out_l4_bytes(uint32_t n) { return chunked(n) * sizeof(rtn_l4ctx_t); }
size_t rtn_out_seqack_bytes(uint32_t n) { return chunked(n) * 8u; }
size_t rtn_out_addr6_bytes(uint32_t n) { return chunked(n) * 24u; }
size_t rtn_out_dlv_bytes(uint32_t n, uint32_t deliver_words) {
  return chunked(n) * (size_t)deliver_words * 8u;
}
static_assert(sizeof(rtn_conn_t) == 8, "rtn_conn_t is 8 bytes");
size_t rtn_out_conn_bytes(uint32_t n) { return chunked(n) * sizeof(rtn_conn_t); }
size_t rtn_out_conn_dlv_bytes(uint32_t n, uint32_t conn_words) { return chunked(n) * conn_words * 8u; }
size_t rtn_out_pd_counts_bytes(uint32_t n, uint32_t n_pd_stmts) {
  return chunked(n) * (n_pd_stmts ? n_pd_stmts : 1u) * sizeof(uint32_t);
}


}  // extern "C"

// ---------------------------------------------------------------------------------------------
// Connection lookup (include/retina_ct.h)

struct rtn_ct {
  int device = 0;
  uint32_t cap = 0, max_live = 0, epoch = 0;
  uint64_t live_bound = 0;   // upper bound of the live connections (exact after a fold)
  uint32_t* table = nullptr;
  uint32_t* occ = nullptr;   // cap bits
  uint32_t* live = nullptr;  // [64] counters, live = their sum (mod 2^32)
  hipModule_t module = nullptr;
  hipFunction_t insert = nullptr, lookup = nullptr, remove = nullptr, clear = nullptr, rehash = nullptr;
  ~rtn_ct() {
    if (table) (void)hipFree(table);
    if (occ) (void)hipFree(occ);
    if (live) (void)hipFree(live);
    if (module) (void)hipModuleUnload(module);
  }
};

namespace {
constexpr uint32_t RTN_CT_CPB = 4;  // chunks per block (one wave each), must match ct_kernel.hip

struct CtArgs {  // must match struct rtn_ct_args in ct_kernel.hip
  const uint64_t* fwd_bm;
  const uint32_t* recs;
  const uint32_t* addr6;
  const uint64_t* conn;
  uint64_t* out;
  uint32_t* table;
  uint32_t* occ;
  uint32_t* live;
  uint32_t n;
  uint32_t cap_mask;
  uint32_t max_live;
  uint32_t epoch;
  uint32_t check;
};

int32_t hip_fail(const char* what, hipError_t e) { return fail(RTN_EDEVICE, std::string(what) + ": " + hipGetErrorString(e)); }

// Exact live count: wait for the stream, sum the 64 counters and fold them into counter 0.
int32_t ct_fold(rtn_ct* ct, hipStream_t s, uint32_t* live_out) {
  uint32_t c[64];
  hipError_t e = s ? hipStreamSynchronize(s) : hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(c, ct->live, sizeof(c), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return hip_fail("ct_fold", e);
  uint32_t sum = 0;
  for (uint32_t v : c) sum += v;
  uint32_t z[64] = {};
  z[0] = sum;
  e = hipMemcpy(ct->live, z, sizeof(z), hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_fail("ct_fold", e);
  ct->live_bound = sum;
  *live_out = sum;
  return RTN_OK;
}

int32_t ct_clear(rtn_ct* ct, uint32_t* table, hipStream_t s) {
  uint32_t cap = ct->cap;
  void* p[] = {&table, &cap};
  hipError_t e = hipModuleLaunchKernel(ct->clear, (cap + 255u) / 256u, 1, 1, 256, 1, 1, 0, s, p, nullptr);
  return e == hipSuccess ? RTN_OK : hip_fail("rtn_ct_clear", e);
}
}  // namespace

extern "C" {

int32_t rtn_ct_create(int device, uint32_t capacity_log2, uint32_t max_connections, rtn_ct_t** out) {
  if (!out) return fail(RTN_EINVAL, "null argument");
  if (capacity_log2 < 6 || capacity_log2 > 30) return fail(RTN_EINVAL, "capacity_log2 must be in [6, 30]");
  std::shared_ptr<std::vector<uint8_t>> code;
  int32_t rc = compile_code_object(env_defines() + ct_template(), code);
  if (rc) return rc;
  auto ct = std::make_unique<rtn_ct>();
  ct->device = device;
  ct->cap = 1u << capacity_log2;
  ct->max_live = max_connections;
  if (hipSetDevice(device) != hipSuccess) return fail(RTN_EDEVICE, "hipSetDevice failed");
  hipError_t e = hipModuleLoadData(&ct->module, code->data());
  if (e != hipSuccess) return hip_fail("hipModuleLoadData", e);
  const char* names[] = {"rtn_ct_insert", "rtn_ct_lookup", "rtn_ct_remove_k", "rtn_ct_clear", "rtn_ct_rehash"};
  hipFunction_t* fns[] = {&ct->insert, &ct->lookup, &ct->remove, &ct->clear, &ct->rehash};
  for (int k = 0; k < 5; ++k) {
    e = hipModuleGetFunction(fns[k], ct->module, names[k]);
    if (e != hipSuccess) return hip_fail("hipModuleGetFunction", e);
  }
  e = hipMalloc(reinterpret_cast<void**>(&ct->table), (size_t)ct->cap * 64u);
  if (e != hipSuccess) return hip_fail("hipMalloc(table)", e);
  e = hipMalloc(reinterpret_cast<void**>(&ct->occ), ct->cap / 8u);
  if (e != hipSuccess) return hip_fail("hipMalloc(occ)", e);
  e = hipMemset(ct->occ, 0, ct->cap / 8u);
  if (e != hipSuccess) return hip_fail("hipMemset(occ)", e);
  e = hipMalloc(reinterpret_cast<void**>(&ct->live), 64 * 4);
  if (e != hipSuccess) return hip_fail("hipMalloc", e);
  e = hipMemset(ct->live, 0, 64 * 4);
  if (e != hipSuccess) return hip_fail("hipMemset", e);
  rc = ct_clear(ct.get(), ct->table, nullptr);
  if (rc) return rc;
  e = hipDeviceSynchronize();
  if (e != hipSuccess) return hip_fail("hipDeviceSynchronize", e);
  *out = ct.release();
  return RTN_OK;
}

int32_t rtn_ct_destroy(rtn_ct_t* ct) {
  delete ct;
  return RTN_OK;
}

int32_t rtn_ct_process(rtn_ct_t* ct, const rtn_pc_out_t* pc, uint32_t n, rtn_ct_entry_t* out, void* stream) {
  if (!ct || !pc || !out) return fail(RTN_EINVAL, "null argument");
  if (n > RTN_MAX_FRAMES) return fail(RTN_EINVAL, "batch larger than RTN_MAX_FRAMES");
  if (n == 0) return RTN_OK;
  if (!pc->fwd_bitmap || !pc->l4 || !pc->conn) return fail(RTN_EINVAL, "rtn_pc_out_t needs fwd_bitmap, l4 and conn");
  if (!pc->addr6) return fail(RTN_EINVAL, "rtn_pc_out_t needs addr6 (IPv6 keys)");
  CtArgs a;
  a.fwd_bm = pc->fwd_bitmap;
  a.recs = reinterpret_cast<const uint32_t*>(pc->l4);
  a.addr6 = reinterpret_cast<const uint32_t*>(pc->addr6);
  a.conn = reinterpret_cast<const uint64_t*>(pc->conn);
  a.out = reinterpret_cast<uint64_t*>(out);
  a.table = ct->table;
  a.occ = ct->occ;
  a.live = ct->live;
  a.n = n;
  a.cap_mask = ct->cap - 1u;
  a.max_live = ct->max_live;
  a.epoch = ++ct->epoch;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // Admission against max_connections on the device: one reservation atomic per block that
  // opens connections (RTN_CT_SPREAD_COUNTERS=1 selects the unchecked variant with spread
  // counters in the experiments build only).
#ifdef RTN_EXPERIMENTS
  static const bool spread = getenv("RTN_CT_SPREAD_COUNTERS") != nullptr;
#else
  const bool spread = false;
#endif
  a.check = spread ? 0u : 1u;
  const uint32_t chunks = (n + RTN_CHUNK_FRAMES - 1u) / RTN_CHUNK_FRAMES;
  void* p[] = {&a};
  const uint32_t blocks = (chunks + RTN_CT_CPB - 1u) / RTN_CT_CPB;
  hipError_t e = hipModuleLaunchKernel(ct->insert, blocks, 1, 1, 64u * RTN_CT_CPB, 1, 1, 0, s, p, nullptr);
  if (e != hipSuccess) return hip_fail("rtn_ct_insert", e);
  e = hipModuleLaunchKernel(ct->lookup, blocks, 1, 1, 64u * RTN_CT_CPB, 1, 1, 0, s, p, nullptr);
  if (e != hipSuccess) return hip_fail("rtn_ct_lookup", e);
  return RTN_OK;
}

int32_t rtn_ct_remove(rtn_ct_t* ct, const uint32_t* slots, uint32_t n, void* stream) {
  if (!ct || (!slots && n)) return fail(RTN_EINVAL, "null argument");
  if (n == 0) return RTN_OK;
  uint32_t mask = ct->cap - 1u;
  uint32_t* table = ct->table;
  uint32_t* occ = ct->occ;
  uint32_t* live = ct->live;
  void* p[] = {&table, &occ, &live, &slots, &n, &mask};
  hipError_t e = hipModuleLaunchKernel(ct->remove, (n + 255u) / 256u, 1, 1, 256, 1, 1, 0,
                                       reinterpret_cast<hipStream_t>(stream), p, nullptr);
  return e == hipSuccess ? RTN_OK : hip_fail("rtn_ct_remove", e);
}

int32_t rtn_ct_rebuild(rtn_ct_t* ct, uint32_t* new_slot, void* stream) {
  if (!ct || !new_slot) return fail(RTN_EINVAL, "null argument");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  uint32_t *dst = nullptr, *docc = nullptr;
  hipError_t e = hipMalloc(reinterpret_cast<void**>(&dst), (size_t)ct->cap * 64u);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&docc), ct->cap / 8u);
  if (e == hipSuccess) e = hipMemsetAsync(docc, 0, ct->cap / 8u, s);
  if (e != hipSuccess) {
    if (dst) (void)hipFree(dst);
    if (docc) (void)hipFree(docc);
    return hip_fail("rtn_ct_rebuild alloc", e);
  }
  int32_t rc = ct_clear(ct, dst, s);
  if (rc) {
    (void)hipFree(dst);
    (void)hipFree(docc);
    return rc;
  }
  const uint32_t* src = ct->table;
  uint32_t mask = ct->cap - 1u;
  void* p[] = {&src, &dst, &docc, &new_slot, &mask};
  e = hipModuleLaunchKernel(ct->rehash, (ct->cap + 255u) / 256u, 1, 1, 256, 1, 1, 0, s, p, nullptr);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    (void)hipFree(dst);
    (void)hipFree(docc);
    return hip_fail("rtn_ct_rehash", e);
  }
  (void)hipFree(ct->table);
  (void)hipFree(ct->occ);
  ct->table = dst;
  ct->occ = docc;
  return RTN_OK;
}

int32_t rtn_ct_stats(rtn_ct_t* ct, rtn_ct_stats_t* st) {
  if (!ct || !st) return fail(RTN_EINVAL, "null argument");
  uint32_t live = 0;
  int32_t rc = ct_fold(ct, nullptr, &live);
  if (rc) return rc;
  st->capacity = ct->cap;
  st->live = live;
  st->epoch = ct->epoch;
  st->max_connections = ct->max_live;
  return RTN_OK;
}

void* rtn_ct_table(rtn_ct_t* ct) { return ct ? ct->table : nullptr; }
size_t rtn_out_ct_bytes(uint32_t n) { return chunked(n) * sizeof(rtn_ct_entry_t); }

}  // extern "C"
