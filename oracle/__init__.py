"""ORACLE — TEST INFRASTRUCTURE ONLY.

A CPU restatement of Retina's packet stage (stanford-esrg/retina, reference snapshot
2025-09-19), used only as the checker by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg. Nothing in retina_amd/ imports it; the product path is the HIP kernel.

Pieces (each cites the reference lines it restates):
  filterlang.py  filter grammar, DNF, fully-qualified patterns, Filter::new, the
                 PacketContinue PTree (build/prune/sort/else-if marking) and a code generator
                 that emits (a) the Rust filtergen would produce (normalised) and (b) C.
  packet.py      Mbuf::get_data bounds, Ethernet/IPv4/IPv6/TCP/UDP parse_from, L4Context::new,
                 Payload::from_mbuf, and a tree evaluator (pure Python; small cases).
  cgen.py        builds the generated C packet_continue + L4Context into a shared library
                 (gcc -O3 -march=native) for large batches and for the CPU baseline.
  pcap.py        libpcap / pcapng readers for the reference's traces/.

Parity pinning (see DESIGN.md "Oracle"): the reference cannot be built here (no cargo/rustc,
DPDK, libpcap) and ships no golden vectors for per-packet parsing, so the oracle is pinned by
(1) the reference's own compiler unit tests (ptree.rs / ast.rs / actions.rs KATs), ported in
tests/, (2) agreement of two independent restatements (this Python oracle vs. the product C++
compiler and HIP kernel, and packet.py vs. the generated C), and (3) committed golden fixtures
built from the reference's traces. Per-packet parse results are "parity unpinned" against a
running reference.
"""
