// rtnc: command-line front end of the filter compiler (the filtergen step, run ahead of time).
//   rtnc <spec.toml> [--tree] [--rust] [--hip]
//   rtnc --filter "<filter>" [--datatype ConnRecord] ...
//   rtnc <spec.toml> --layers      every FilterLayer's collapsed tree (filtergen/src/lib.rs:274-304)
//   rtnc <spec.toml> --deliver     the PacketDeliver filter: tree, facts, Rust listing, HIP body
#include <cstdio>
#include <fstream>
#include <iostream>
#include <sstream>

#include "codegen.hpp"

int main(int argc, char** argv) {
  std::vector<rtn::SubscriptionSpec> subs;
  bool tree = false, rust = false, hip = false, layers = false, deliver = false;
  std::string filter;
  std::vector<std::string> dts;
  std::string spec_path;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--tree") tree = true;
    else if (a == "--rust") rust = true;
    else if (a == "--hip") hip = true;
    else if (a == "--layers") layers = true;
    else if (a == "--deliver") deliver = true;
    else if (a == "--filter" && i + 1 < argc) filter = argv[++i];
    else if (a == "--datatype" && i + 1 < argc) dts.push_back(argv[++i]);
    else spec_path = a;
  }
  if (!tree && !rust && !hip && !layers && !deliver) tree = rust = true;
  try {
    if (!spec_path.empty()) {
      std::ifstream f(spec_path);
      if (!f) {
        fprintf(stderr, "cannot open %s\n", spec_path.c_str());
        return 2;
      }
      std::stringstream ss;
      ss << f.rdbuf();
      subs = rtn::parse_subscription_toml(ss.str());
    } else {
      rtn::SubscriptionSpec s(filter, "cb");
      if (dts.empty()) dts.push_back("ConnRecord");
      for (auto& d : dts) {
        rtn::DataType dt;
        if (!rtn::lookup_datatype(d, dt)) throw rtn::FilterError("Invalid datatype: " + d);
        s.add_datatype(dt);
      }
      subs.push_back(s);
    }
    if (layers) {
      for (auto l : {rtn::FilterLayer::PacketContinue, rtn::FilterLayer::Packet, rtn::FilterLayer::Protocol,
                     rtn::FilterLayer::Session, rtn::FilterLayer::ConnectionDeliver, rtn::FilterLayer::PacketDeliver})
        std::cout << rtn::filter_subtree(l, subs).pprint();
      return 0;
    }
    auto prog = rtn::compile_packet_program(subs);
    if (tree) std::cout << prog.tree.pprint();
    if (rust) std::cout << prog.rust_listing;
    if (hip) std::cout << prog.hip_body;
    if (deliver) {
      std::cout << prog.pd_tree.pprint();
      for (size_t k = 0; k < prog.pd_facts.size(); ++k)
        std::cout << "fact " << k << ":" << (prog.pd_facts[k].kind == rtn::PdFact::Service ? " service " : " session ") << prog.pd_facts[k].pred
                  << "\n";
      std::cout << prog.rust_pd_listing << prog.hip_pd_body;
    }
  } catch (const rtn::FilterError& e) {
    fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
  return 0;
}
