"""Timing variants of retina_amd/csrc/kernels/pc_kernel.hip, made by text patches (tools/README.md).
Each variant is a function src -> src; `base` is the product kernel unchanged."""
from __future__ import annotations

from pathlib import Path

KERNEL = Path(__file__).resolve().parent.parent / "retina_amd" / "csrc" / "kernels" / "pc_kernel.hip"


def _sub(src: str, old: str, new: str) -> str:
    assert old in src, f"variant patch does not apply: {old[:60]!r}"
    return src.replace(old, new)


def base(src: str) -> str:
    return src


def ceiling(src: str) -> str:
    """A fully coalesced 16-B-per-lane read of the head slab (+ ext for split): the HBM read
    ceiling of the same bytes. Writes nothing."""
    body = '''{
  const rtn_u64 n16 = (rtn_u64)a.n * a.stride / 16u;
  const rtn_v4u* p = reinterpret_cast<const rtn_v4u*>(a.slab);
  rtn_u32 x = 0;
  for (rtn_u64 k = blockIdx.x * (rtn_u64)blockDim.x + threadIdx.x; k < n16; k += (rtn_u64)gridDim.x * blockDim.x) {
    const rtn_v4u v = __builtin_nontemporal_load(p + k);
    x ^= v.x + v.y + v.z + v.w;
  }
  if (x == 0x9E3779B9u) a.counters[3] = x;
}'''
    for k in ("rtn_pc_kernel(rtn_args a) { rtn_run<RTN_MONO, false>(a); }",
              "rtn_pc_kernel_s64(rtn_args a) { rtn_run<RTN_S64, false>(a); }",
              "rtn_pc_kernel_split(rtn_args a) { rtn_run<RTN_SPLIT, false>(a); }",
              "rtn_pc_kernel_splitc(rtn_args a) { rtn_run<RTN_SPLITC, false>(a); }"):
        src = _sub(src, k, k.split(" {")[0] + " " + body)
    return src


def nostores(src: str) -> str:
    """Everything but the record / IPv6-address / delivery stores (bitmaps still written)."""
    src = _sub(src, "  if (fwd) {\n    const rtn_u32 r", "  if (fwd && a.n == 0u) {\n    const rtn_u32 r")
    src = _sub(src, "    if (d) {", "    if (d && a.n == 0u) {")
    src = _sub(src, "  const bool six = fwd && v.v6 && (a.flags & 1u);", "  const bool six = false;")
    src = _sub(src, "    rtn_flush<CONN>(a, ring, cring, ch, lane, ch.nrec - ch.nflushed);", "")
    src = _sub(src, "    if (ch.ntcp != ch.ntflushed) rtn_flush_t4(a, ring4, ch, lane, ch.ntcp - ch.ntflushed);", "")
    src = _sub(src, "  if (fr || ft) {", "  if (false) {")
    return src


VARIANTS = {"base": base, "ceiling": ceiling, "nostores": nostores}


def dense(src: str) -> str:
    """Timing only: a chunk's records go to one dense 128-record region (chunk * 128 + k, no block
    interleave; chunks with more than 128 records overlap their neighbours)."""
    src = _sub(src, "rtn_v4u* dst = reinterpret_cast<rtn_v4u*>(a.recs + rtn_rec_slot(nch, c, ch.nflushed));",
               "rtn_v4u* dst = reinterpret_cast<rtn_v4u*>(a.recs + ch.rec_base / 2u + ch.nflushed);")
    return _sub(src, "if (lane < nl) RTN_ST(dst + (lane / RTN_RB) * nch * RTN_RB + lane % RTN_RB, src[lane]);",
                "if (lane < nl) RTN_ST(dst + lane, src[lane]);")


def nobitmaps(src: str) -> str:
    """Timing only: no pc / fwd bitmap stores."""
    src = _sub(src, "      RTN_ST8(a.pc_bm + gb + lane, ch.my_pc);\n", "")
    return _sub(src, "      RTN_ST8(a.fwd_bm + gb + lane, ch.my_fwd);\n", "")


def bm128(src: str) -> str:
    """Timing only: the pc and fwd words of a chunk leave as one whole 128-B line (into the pc
    bitmap, two chunks per line: overlapping)."""
    src = _sub(src, "      RTN_ST8(a.pc_bm + gb + lane, ch.my_pc);\n      RTN_ST8(a.fwd_bm + gb + lane, ch.my_fwd);",
               "      RTN_ST8(a.pc_bm + (gb & ~15u) + lane, ch.my_pc);\n    }\n    if (lane >= 8u && lane < 16u) {\n"
               "      RTN_ST8(a.pc_bm + (gb & ~15u) + lane, __shfl(ch.my_fwd, (int)(lane - 8u)));")
    return src


def noext(src: str) -> str:
    """Timing only: the bytes past 64 are never fetched (frames that need them parse zeros)."""
    return _sub(src, "const bool need = rtn_need_hi(lo, dl);", "const bool need = rtn_need_hi(lo, dl) && a.n == 0u;")


def tstores(src: str) -> str:
    """Record-block stores through the caches (plain) instead of non-temporal."""
    return _sub(src, "#define RTN_ST(p, v) __builtin_nontemporal_store((v), (p))", "#define RTN_ST(p, v) (*(p) = (v))")


def _store_asm(mods: str):
    def v(src: str) -> str:
        return _sub(src, "#define RTN_ST(p, v) __builtin_nontemporal_store((v), (p))",
                    '#define RTN_ST(p, v) asm volatile("global_store_dwordx4 %0, %1, off ' + mods +
                    '" ::"v"(p), "v"(v) : "memory")')
    v.__doc__ = f"Record-block stores as global_store_dwordx4 ... {mods}."
    return v


def dm_opq(src: str) -> str:
    """Delivery bits as an opaque 0/1 shifted into its half-word (v_cndmask with inline 0/1, then
    v_lshl_or with an inline shift): no 1 << b constant held in a register across the loop."""
    return _sub(src, "#define RTN_DM_SET(m, w, b, r) ((m)[w] |= (r) ? (1ull << (b)) : 0ull)",
                "__device__ __forceinline__ rtn_u32 rtn_opq(rtn_u32 x) { asm(\"\" : \"+v\"(x)); return x; }\n"
                "#define RTN_DM_SET(m, w, b, r) ((m)[w] |= (rtn_u64)(rtn_opq((r) ? 1u : 0u) << ((b) % 32u)) << ((b) / 32u * 32u))")


def oldform(src: str) -> str:
    """The compact ext path as a run-time branch of the split kernel instance (round-2 form)."""
    src = _sub(src, "rtn_pc_kernel_splitc(rtn_args a) { rtn_run<RTN_SPLITC, false>(a); }",
               "rtn_pc_kernel_splitc(rtn_args a) { rtn_run<RTN_SPLIT, false>(a); }")
    return _sub(src, "        if (MODE == RTN_SPLITC) {\n          const rtn_u64 nm = __ballot(need);",
                "        if (MODE == RTN_SPLIT && (a.flags & 16u)) {\n          const rtn_u64 nm = __ballot(need);")


def splitc_w4(src: str) -> str:
    """The compact split kernel held to 4 waves per SIMD (<= 128 VGPRs)."""
    return _sub(src, "extern \"C\" __global__ void __launch_bounds__(256) rtn_pc_kernel_splitc(",
                "extern \"C\" __global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) rtn_pc_kernel_splitc(")


def splitc_pf(src: str) -> str:
    """The compact split kernel also keeps the next group's head loads in flight."""
    return _sub(src, "constexpr bool prefetch = MODE == RTN_S64;", "constexpr bool prefetch = MODE == RTN_S64 || MODE == RTN_SPLITC;")


VARIANTS.update({"oldform": oldform, "splitc_w4": splitc_w4, "splitc_pf": splitc_pf, "dm_opq": dm_opq, "dense": dense, "nobitmaps": nobitmaps, "bm128": bm128, "noext": noext, "tstores": tstores,
                 "st_sc1": _store_asm("sc1"), "st_sc0sc1": _store_asm("sc0 sc1"),
                 "st_ntsc1": _store_asm("nt sc1"), "st_nt": _store_asm("nt")})


def chunk512(src: str) -> str:
    """Timing only: 512-frame chunks (the round-2 layout before 256; the compact layout needs
    #compact512). Run with @GRID = ceil(n / 2048) blocks so that every chunk gets its own wave."""
    return _sub(src, "#define RTN_CHUNK_GROUPS 4u", "#define RTN_CHUNK_GROUPS 8u")


def chunk128(src: str) -> str:
    """Timing only: 128-frame chunks (@GRID = ceil(n / 512) blocks)."""
    return _sub(src, "#define RTN_CHUNK_GROUPS 4u", "#define RTN_CHUNK_GROUPS 2u")


def rb128(src: str) -> str:
    """Timing only: 128-record blocks (a 512-frame chunk's records in 4 interleaved streams)."""
    return _sub(src, "#define RTN_RB 64u", "#define RTN_RB 128u")


def wpb2(src: str) -> str:
    """Per-block LDS sized for 2 waves (run with RTN_BLOCK=128: 128-thread blocks, one chunk per
    wave as before, so a block retires after 2 chunks instead of 4)."""
    for arr in ("rtn_ring[4]", "rtn_ring4[4]", "rtn_cring[4]", "rtn_ring6[4]", "rtn_tile[4]"):
        src = _sub(src, arr, arr.replace("[4]", "[2]"))
    return src


def kz(src: str) -> str:
    """Predicate constants XORed with a per-group run-time zero (readfirstlane(nrec >> 31)) so that
    the compiler cannot hoist them out of the group loop into SGPRs (cfg4: 72 SGPR spills)."""
    src = _sub(src, "#ifndef RTN_K\n", "#define RTN_K(c) ((c) ^ rtn_kz)\n#define RTN_KZ_DECL(x) const rtn_u32 rtn_kz = (x).kz;\n#ifndef RTN_K\n")
    src = _sub(src, "struct rtn_view {\n", "struct rtn_view {\n  rtn_u32 kz;\n")
    src = _sub(src, "struct rtn_cview {\n", "struct rtn_cview {\n  rtn_u32 kz;\n")
    src = _sub(src, "  rtn_parse<NW>(w, dl, v);\n", "  rtn_parse<NW>(w, dl, v);\n  v.kz = __builtin_amdgcn_readfirstlane(ch.nrec >> 31);\n")
    src = _sub(src, "      c.v6 = v.v6;\n", "      c.v6 = v.v6;\n      c.kz = v.kz;\n")
    src = _sub(src, "      c.v6 = v6;\n", "      c.v6 = v6;\n      c.kz = 0u;\n")
    return src


def kzdm(src: str) -> str:
    """kz, and the statement-mask bits (1 << b) XORed with the same zero."""
    src = kz(src)
    return _sub(src, "#define RTN_DM_SET(m, w, b, r) ((m)[w] |= (r) ? (1ull << (b)) : 0ull)",
                "#define RTN_DM_SET(m, w, b, r) ((m)[w] |= (r) ? ((1ull << (b)) ^ (rtn_u64)rtn_kz) : 0ull)")


VARIANTS.update({"kz": kz, "kzdm": kzdm, "chunk512": chunk512, "chunk128": chunk128, "rb128": rb128, "wpb2": wpb2})


def nobarrel(src: str) -> str:
    """Timing only: every wave takes the Eth/IPv4 constant-offset extraction (wrong views for
    lanes with other offsets): the cost of the per-lane barrel shifter."""
    return _sub(src, "    rtn_extract_v<NW>(w, q, v.l4off, v);", "    rtn_extract_c<NW, 14, 34>(w, v);")


def nofilter(src: str) -> str:
    """Timing only: the generated filter is replaced by "accept every IP frame, deliver one
    statement on half of them" (a destination-address bit), keeping the output volume."""
    return _sub(src, "  rtn_filter(v, act, dm);", "  act = (v.v4 || v.v6) ? 1u : 0u; dm[0] = (v.v4 || v.v6) ? (v.l3w[4] & 1u) : 0u;")


VARIANTS.update({"nobarrel": nobarrel, "nofilter": nofilter})


def dm32(src: str) -> str:
    """Statement bits set on the 32-bit half that holds them (no 64-bit OR chain whose high
    half ORs zeros)."""
    return _sub(src, "#define RTN_DM_SET(m, w, b, r) ((m)[w] |= (r) ? (1ull << (b)) : 0ull)",
                "#define RTN_DM_SET(m, w, b, r) (reinterpret_cast<rtn_u32*>(m)[2 * (w) + ((b) >> 5)] |= (r) ? (1u << ((b) & 31)) : 0u)")


VARIANTS.update({"dm32": dm32})


def withconn(src: str) -> str:
    """The kernels without the connection stage compiled as before its specialisation: the stage's
    code and LDS ring present, skipped at run time (flags bit 2)."""
    src = src.replace("if (CONN) {", "if (CONN && (a.flags & 4u)) {")
    for m in ("RTN_MONO", "RTN_S64", "RTN_SPLIT", "RTN_SPLITC"):
        src = _sub(src, f"{{ rtn_run<{m}, false>(a); }}", f"{{ rtn_run<{m}, true>(a); }}")
    return src


VARIANTS.update({"withconn": withconn})


def not4(src: str) -> str:
    """Timing only: no TCP seq/ack side stream (the seqack ring and its stores)."""
    return _sub(src, "const bool t4 = fwd && v.tcp && (a.flags & 32u);", "const bool t4 = false;")


def pad128(src: str) -> str:
    """Chunk-end stores padded to whole 128-B lines (the round-2 form) instead of 64-B requests:
    records to 8, seq/ack entries to 16, IPv6 address bytes to 128. (As pad64 against the 128-B
    form, in-process on one box: cfg4 0.1671 -> 0.1655 ms, cfg3 and cfg2 unchanged.)"""
    src = _sub(src, "  const rtn_u32 nl = (nrecs + 3u) & ~3u;", "  const rtn_u32 nl = (nrecs + 7u) & ~7u;")
    src = _sub(src, "  const rtn_u32 nl = ((nent + 1u) / 2u + 3u) & ~3u;", "  const rtn_u32 nl = ((nent + 1u) / 2u + 7u) & ~7u;")
    return _sub(src, "  const rtn_u32 nu = ((nent * 24u + 63u) & ~63u) / 16u;", "  const rtn_u32 nu = ((nent * 24u + 127u) & ~127u) / 16u;")


def noq6(src: str) -> str:
    """Waves mixing the four common stacks take the barrel shifter (the round-2 form) instead of
    rtn_extract_q6."""
    return _sub(src, "  } else if (__ballot(ip && v.l4off != v.l3off + (v.v6 ? 40u : 20u)) == 0ull) {",
                "  } else if (false) {")


def t4dense(src: str) -> str:
    """Timing only: a chunk's seq/ack entries dense per chunk (chunk * 256 + TCP rank, like
    addr6) instead of in RTN_REC_INDEX blocks: one contiguous run per chunk."""
    return _sub(src, "  if (lane < nl) RTN_ST(dst + (lane / (RTN_RB / 2u)) * nch * (RTN_RB / 2u) + lane % (RTN_RB / 2u), src[lane]);\n}\n\n// IPv6",
                "  (void)dst;\n  rtn_v4u* dd = reinterpret_cast<rtn_v4u*>(a.seqack + ch.rec_base + ch.ntflushed);\n"
                "  if (lane < nl) RTN_ST(dd + lane, src[lane]);\n}\n\n// IPv6")


def recdense(src: str) -> str:
    """Timing only: a chunk's records dense per chunk (chunk * 256 + rank) instead of in
    RTN_REC_INDEX blocks (the connection-stage entries stay interleaved)."""
    return _sub(src, "  if (lane < nl) RTN_ST(dst + (lane / RTN_RB) * nch * RTN_RB + lane % RTN_RB, src[lane]);",
                "  (void)dst;\n  rtn_v4u* dd = reinterpret_cast<rtn_v4u*>(a.recs + ch.rec_base + ch.nflushed);\n"
                "  if (lane < nl) RTN_ST(dd + lane, src[lane]);")


def dmsb(src: str) -> str:
    """A scheduling barrier after every statement-mask bit of the generated filter: the compiler
    cannot hoist later predicates' compares above it (their lane masks stay out of SGPRs until
    needed)."""
    src = _sub(src, "#define RTN_DM_SET(m, w, b, r) ((m)[w] |= (r) ? (1ull << (b)) : 0ull)",
               "#define RTN_DM_SET(m, w, b, r) do { (m)[w] |= (r) ? (1ull << (b)) : 0ull; __builtin_amdgcn_sched_barrier(0); } while (0)")
    return _sub(src, "#define RTN_DM_SETV(m, w, b, r) ((m)[w] |= (r) ? (1ull << (b)) : 0ull)",
                "#define RTN_DM_SETV(m, w, b, r) do { (m)[w] |= (r) ? (1ull << (b)) : 0ull; __builtin_amdgcn_sched_barrier(0); } while (0)")


def ksb(src: str) -> str:
    """A scheduling barrier at every predicate constant of the generated filter: predicates are
    evaluated in program order."""
    return _sub(src, "#ifndef RTN_K\n", "#define RTN_K(c) (__builtin_amdgcn_sched_barrier(0), (c))\n#ifndef RTN_K\n")



VARIANTS.update({"not4": not4, "pad128": pad128, "noq6": noq6, "t4dense": t4dense, "recdense": recdense,
                 "dmsb": dmsb, "ksb": ksb})


def nodlv(src: str) -> str:
    """Timing only: no delivery-record stores (the dlv bitmap is still written)."""
    return _sub(src, "    if (d) {\n      const rtn_u64 slot_i", "    if (d && a.n == 0u) {\n      const rtn_u64 slot_i")


def dlvnt(src: str) -> str:
    """Delivery records stored non-temporally instead of through the caches (8-B stores at the
    record's rank)."""
    return _sub(src, "      for (int j = 0; j < RTN_DELIVER_WORDS; ++j) RTN_ST8(dp + j, dm[j]);",
                "      for (int j = 0; j < RTN_DELIVER_WORDS; ++j) __builtin_nontemporal_store(dm[j], dp + j);")


VARIANTS.update({"nodlv": nodlv, "dlvnt": dlvnt})


def write(name: str, outdir: Path) -> Path:
    """A variant file: a '+'-joined list of VARIANTS applied to the current kernel, or
    'file=<path>' (a kernel source as is, e.g. an older revision: git show REV:path > file)."""
    outdir.mkdir(parents=True, exist_ok=True)
    if name.startswith("file="):
        return Path(name[5:]).resolve()
    spec = name.split("+")
    src = KERNEL.read_text()
    for s in spec:
        src = VARIANTS[s](src)
    p = outdir / f"pc_kernel_{name.replace('+', '_')}.hip"
    p.write_text(src)
    return p
