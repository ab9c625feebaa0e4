/*
 * retina_pc.h — C ABI of the MI355X packet-stage filter (drop-in for Retina's packet stage).
 *
 * Replaces, per batch of mbufs, what the reference does per mbuf:
 *   - Subscription::continue_packet            core/src/subscription/mod.rs:125-127
 *     -> the filtergen-generated packet_continue(mbuf, core_id) -> Actions
 *        (type PacketContFn, core/src/filter/mod.rs:49; emitted at filtergen/src/lib.rs:336-339)
 *   - the PacketContinue gate + L4Context::new in Subscription::process_packet
 *                                              core/src/subscription/mod.rs:94-116,
 *                                              core/src/conntrack/pdu.rs:86-171
 *   - packet-level callbacks fired inside packet_continue (ZcFrame / Payload subscriptions,
 *     filtergen/src/data.rs:299-331), reported as per-packet "statement masks" that name the
 *     callback sites in generated-code order; the host invokes the callbacks.
 *   - filtergen itself (filtergen/src/lib.rs:241-385, packet layer): rtn_program_compile turns a
 *     subscription spec (the #[subscription("spec.toml")] TOML format, filtergen/src/parse.rs)
 *     into a tree-specialised HIP kernel.
 *   - optional connection stage of each forwarded frame (rtn_conn_t): the ConnId the conntrack
 *     table is keyed by (conntrack/conn_id.rs:111-117) as a hash + orientation, whether the frame
 *     may open a connection (Conn::new_tcp / new_udp, conntrack/conn/mod.rs:53-96), and the
 *     generated first-packet `packet_filter` (FilterLayer::Packet, filtergen/src/lib.rs:284-285)
 *     that ConnInfo::filter_first_packet runs for a new connection (conn/conn_info.rs:42-50).
 * The reference callers are core/src/lcore/rx_core.rs:117-141 (online) and
 * core/src/runtime/offline.rs:67-82 (pcap). See INTEGRATION.md for the Rust extern "C" binding.
 *
 * Conventions: every function returns 0 on success or a negative errno-style code; the message
 * of the last failure on the calling thread is available from rtn_last_error(). No C++
 * exceptions cross this boundary. Pointers in rtn_batch_t / rtn_pc_out_t are device pointers
 * (hipMalloc'd) unless stated. A context is thread-compatible, not thread-safe: use one per
 * RX thread/stream (like the reference's per-lcore Subscription use).
 */
#ifndef RETINA_PC_H
#define RETINA_PC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTN_OK 0
#define RTN_EINVAL (-22)   /* bad argument or layout */
#define RTN_EFILTER (-74)  /* filter / subscription spec rejected (what filtergen would refuse) */
#define RTN_EDEVICE (-5)   /* HIP runtime or device failure */
#define RTN_ECOMPILE (-38) /* kernel compilation (hiprtc) failed */
#define RTN_ERANGE (-34)   /* output buffer too small */

typedef struct rtn_program rtn_program_t; /* compiled subscription set (host only)        */
typedef struct rtn_pc rtn_pc_t;           /* program loaded on one device, ready to run  */

/* Compacted L4Context of a forwarded packet (PacketContinue && L4Context::new Ok), 16 bytes.
 * Together with its side streams it holds every field of conntrack/pdu.rs:66-84, and no field
 * that is always zero for the record's kind:
 *   IPv4 TCP: w0 = src, w1 = dst (u32::from(Ipv4Addr), host order); seq_no | ack_no << 32 in seqack
 *   IPv4 UDP: w0 = src, w1 = dst                                       (seq_no = ack_no = 0)
 *   IPv6 TCP: w0|w1 = src bytes 0..7 (memory order); src bytes 8..15 | dst in addr6 (24 B);
 *             seq_no | ack_no << 32 in seqack
 *   IPv6 UDP: w0|w1 = src bytes 0..7; src bytes 8..15 | dst in addr6   (seq_no = ack_no = 0)
 * The frame a record belongs to is implied by its position (see rtn_pc_out_t). */
typedef struct rtn_l4ctx {
  uint32_t w0;
  uint32_t w1;
  uint32_t ports;   /* src_port | dst_port << 16                                         */
  uint32_t meta;    /* RTN_L4_* accessors below: offset, proto, ip version, flags, length */
} rtn_l4ctx_t;

/* L4Context.offset is always 2 mod 4 (14/18-byte L2 + 4*IHL or 40 + 4*doff or 8), so it is
 * stored as offset >> 2 in 6 bits. */
#define RTN_L4_OFFSET(m) ((((m) & 0x3Fu) << 2) | 2u)            /* L4Context.offset           */
#define RTN_L4_PROTO(m) (((m) & 0x40u) ? 17u : 6u)                 /* L4Context.proto            */
#define RTN_L4_IPV6(m) (((m) >> 7) & 1u)                           /* IPv6 (w0|w1 + addr6)       */
#define RTN_L4_FLAGS(m) (((m) >> 8) & 0xFFu)                       /* L4Context.flags (TCP)      */
#define RTN_L4_LENGTH(m) ((m) >> 16)                               /* L4Context.length           */
/* seq_no | ack_no << 32 of a TCP record, in rtn_pc_out_t.seqack */
#define RTN_SEQACK_SEQ(t) ((uint32_t)(t))
#define RTN_SEQACK_ACK(t) ((uint32_t)((t) >> 32))

/* Connection stage of a forwarded frame (8 bytes, indexed like its rtn_l4ctx_t):
 *   hash  = rtn_conn_hash of the canonical ConnId: MurmurHash3-x86-32 block + finaliser steps,
 *           seed 0x5EED, over the words [max ip (4 or 16 B as big-endian u32 words, most
 *           significant first)], [min ip], (max port << 16 | min port), (proto | 0x100 if IPv6),
 *           then h ^= 16 (IPv4) or 40 (IPv6) and fmix32. max/min are Rust's SocketAddr order
 *           (ip, then port), as ConnId::new's cmp::max/min.
 *   info  = packet_filter Actions.data (13 bits) | terminal_actions << 13 | creates << 26 |
 *           src_is_max << 27 | any first-packet statement fired << 28 | IPv6 << 29 | UDP << 30
 *           (the last two repeat the record's, so later stages can skip the record). `creates`: the frame would
 *           open a connection on a table miss (TCP SYN without ACK/RST, or any UDP). The
 *           packet_filter result is that of this frame, which the host uses only when the frame
 *           does open a connection. */
typedef struct rtn_conn {
  uint32_t hash;
  uint32_t info;
} rtn_conn_t;
#define RTN_CONN_PF_DATA(i) ((i) & 0x1FFFu)
#define RTN_CONN_PF_TERMINAL(i) (((i) >> 13) & 0x1FFFu)
#define RTN_CONN_CREATES(i) (((i) >> 26) & 1u)
#define RTN_CONN_SRC_IS_MAX(i) (((i) >> 27) & 1u)
#define RTN_CONN_PF_STMTS(i) (((i) >> 28) & 1u)
#define RTN_CONN_IPV6(i) (((i) >> 29) & 1u) /* the record is IPv6 (its addresses are in addr6)  */
#define RTN_CONN_UDP(i) (((i) >> 30) & 1u)  /* L4Context.proto is UDP (else TCP)              */

/* Largest batch rtn_pc_run accepts (frame indices stay 32-bit inside the kernels). */
#define RTN_MAX_FRAMES (1u << 31)

/* rtn_batch_t.flags */
#define RTN_BATCH_DL_LE64 1u   /* the caller asserts data_len[i] <= 64 for every frame (see below) */
#define RTN_BATCH_EXT_COMPACT 2u /* split layout with ext rows only for the frames that need them  */

/* Status bits (counters[3], rtn_pc_take_status): frames whose results are not the reference's. */
#define RTN_STATUS_HDR_PAST_SLOT 1u /* 64-B slots, no ext: an IP frame's headers run past byte 64 */
#define RTN_STATUS_DL_PAST_SLOT 2u  /* RTN_BATCH_DL_LE64 asserted, but a frame has data_len > 64  */
#define RTN_STATUS_EXT_ROWS 4u      /* RTN_BATCH_EXT_COMPACT: a needed ext row is past ext_rows     */

/* A batch of frames laid out for coalesced HBM reads, in one of two layouts:
 *  - monolithic (ext == NULL): slot i (stride bytes, a multiple of 64) holds the first
 *    min(data_len[i], stride) bytes of frame i;
 *  - split (ext != NULL, stride == 64): slab slot i holds bytes [0, 64) of frame i and ext slot i
 *    (64 bytes) bytes [64, 128). The kernel reads ext[i] only for frames whose headers run past
 *    byte 64 (IPv6, IPv4 options, VLAN + options), so a frame costs 64 B of HBM reads unless it
 *    needs more -- a 128-byte monolithic slot costs a whole 128-B line for every frame.
 * 64-byte slots without ext hold every header only when no frame's headers pass byte 64. The
 * caller must make that checkable: either every data_len is <= 64 and flags has
 * RTN_BATCH_DL_LE64 (a frame cannot be parsed past its data_len, so the slot holds everything
 * the parse reads), or counters is passed so that the status word reaches the caller. Otherwise
 * rtn_pc_run refuses the batch (RTN_EINVAL). A frame that breaks the layout is reported in
 * counters[3] (RTN_STATUS_*) and, when counters is NULL, in the context's sticky status word
 * (rtn_pc_take_status). */
typedef struct rtn_batch {
  const uint8_t* slab;
  uint64_t stride;
  const uint16_t* data_len; /* Mbuf::data_len of each frame (mbuf.rs:95-97) */
  uint32_t n;               /* <= RTN_MAX_FRAMES                                          */
  uint32_t core_id;         /* the calling lcore (passed to CoreId callbacks by the host) */
  const uint8_t* ext;       /* split layout: bytes [64, 128) of each frame, 64-byte slots */
  uint32_t flags;           /* RTN_BATCH_*                                                */
  uint32_t ext_rows;        /* RTN_BATCH_EXT_COMPACT: rows in ext                         */
  const uint32_t* ext_chunk; /* RTN_BATCH_EXT_COMPACT: [ceil(n/256)] row of the first frame of
                                each 256-frame chunk that needs one (an exclusive prefix sum) */
} rtn_batch_t;

/* The compact split layout (RTN_BATCH_EXT_COMPACT): ext holds bytes [64, 128) only of the frames
 * for which rtn_ext_needed() holds, one 64-byte row each, in frame order; the kernel finds frame
 * i's row as ext_chunk[i / RTN_CHUNK_FRAMES] + (number of such frames of the chunk before i).
 * A 128-byte HBM line then carries two needed rows instead of a needed and an unneeded one.
 * The rule is the kernel's own (the frame's headers may pass byte 64 and the frame is longer):
 * `head` is the frame's first 64 bytes (the head slot). A row past ext_rows is not read
 * (RTN_STATUS_EXT_ROWS). */
static inline int rtn_ext_needed(const uint8_t* head, uint16_t data_len) {
  const unsigned et = ((unsigned)head[12] << 8) | head[13];
  const int q = et == 0x8100u;
  const unsigned inner = q ? (((unsigned)head[16] << 8) | head[17]) : et;
  const unsigned ihl4 = (unsigned)(head[q ? 18 : 14] & 0xFu) << 2;
  const unsigned l4 = (q ? 18u : 14u) + (inner == 0x86DDu ? 40u : ihl4);
  const int ip = inner == 0x0800u || inner == 0x86DDu;
  return ip && data_len > 64u && l4 + 20u > 64u;
}

/* Records are ranked per chunk of RTN_CHUNK_FRAMES frames, in frame order: the k-th forwarded
 * frame of chunk c = i / RTN_CHUNK_FRAMES (k = popcount of fwd_bitmap over the chunk's frames
 * before it) has its L4Context at l4[RTN_REC_INDEX(n, c, k)]; conn, conn_dlv, the connection
 * table's rtn_ct_entry_t and the PacketDeliver counts use the same index. A chunk's records sit
 * in blocks of RTN_REC_BLOCK, block j of chunk c at block slot j * nchunks + c, so the chunks'
 * first blocks form one dense stream, their second blocks the next, and so on (the stores of a
 * partly-forwarded batch stay dense).
 * The j-th forwarded IPv6 frame of chunk c (records with RTN_L4_IPV6) has the rest of its
 * addresses (source bytes 8..15, destination) at addr6[c * RTN_CHUNK_FRAMES + j]; dlv_records are
 * ranked by dlv_bitmap the same way (dense per chunk). The j-th TCP record of chunk c (not UDP)
 * has its seq/ack at seqack[RTN_REC_INDEX(n, c, j)]. Bitmaps hold bit i % 64 of word i / 64. */
#define RTN_CHUNK_FRAMES 256u
#define RTN_REC_BLOCK 64u
#define RTN_REC_INDEX(n, chunk, k)                                                             \
  (((uint64_t)((k) / RTN_REC_BLOCK) * (((uint64_t)(n) + RTN_CHUNK_FRAMES - 1u) / RTN_CHUNK_FRAMES) + \
    (uint64_t)(chunk)) * RTN_REC_BLOCK + (uint64_t)((k) % RTN_REC_BLOCK))
/* l4, addr6, conn and seqack must be 16-byte aligned (RTN_EINVAL otherwise). */
typedef struct rtn_pc_out {
  uint64_t* pc_bitmap;   /* [ceil(n/64)]  Actions.data contains PacketContinue               */
  uint64_t* fwd_bitmap;  /* [ceil(n/64)]  ... and L4Context::new succeeded (goes to conntrack) */
  rtn_l4ctx_t* l4;       /* [ceil(n/256)*256] (rtn_out_l4_bytes) at RTN_REC_INDEX; unused slots undefined */
  uint8_t* addr6;        /* optional [ceil(n/256)*256][24] (rtn_out_addr6_bytes): source bytes 8..15
                          and destination of the IPv6 records (raw); a chunk's last store is
                          padded to whole 64-B write requests, so it may write up to 2 entries
                          past the chunk's last IPv6 record (inside the chunk's 256 entries) */
  uint64_t* dlv_bitmap;  /* [ceil(n/64)] frames with >= 1 packet-level callback (if any)     */
  uint64_t* dlv_records; /* [ceil(n/256)*256][deliver_words]: statement mask; the frame is the
                          record's rank among its chunk's dlv_bitmap bits (as for l4)        */
  uint32_t* counters;    /* optional [16] (RTN_COUNTERS_BYTES = 64 B, 8-B aligned), zeroed per run
                          (NULL: no totals, no memset -- one kernel launch); RTN_CNT_* below */
  rtn_conn_t* conn;      /* optional [ceil(n/256)*256]: connection stage, indexed like l4       */
  uint64_t* conn_dlv;    /* [ceil(n/256)*256][conn_words] first-packet statement masks; required
                          with conn when the program has first-packet statements           */
  uint64_t* seqack;      /* optional [ceil(n/256)*256] (rtn_out_seqack_bytes): seq_no | ack_no << 32
                          of the TCP records, IPv4 and IPv6 (NULL: not written)             */
} rtn_pc_out_t;

/* The counters block (u32 word offsets; the byte sums are u64 over two words). The stats names
 * are the reference's thread-local counters (core/src/stats/mod.rs:9-27) as rx_core.rs:127-139
 * and Subscription::process_packet (subscription/mod.rs:102-111) update them per frame. */
#define RTN_COUNTERS_BYTES 64u
#define RTN_CNT_PC 0u          /* u32: Actions.data has PacketContinue (TOTAL_PKT - IGNORED_BY_PACKET_FILTER_PKT) */
#define RTN_CNT_FWD 1u         /* u32: ... and L4Context::new Ok (frames handed to conntrack)  */
#define RTN_CNT_DLV 2u         /* u32: frames with >= 1 packet-level callback                  */
#define RTN_CNT_STATUS 3u      /* u32: RTN_STATUS_* bits                                       */
#define RTN_CNT_TOTAL_BYTE 4u  /* u64: TOTAL_BYTE (data_len of every frame)                    */
#define RTN_CNT_IGNORED_BYTE 6u /* u64: IGNORED_BY_PACKET_FILTER_BYTE                          */
#define RTN_CNT_TCP_PKT 8u     /* u32: TCP_PKT (forwarded, L4Context.proto == 6)               */
#define RTN_CNT_UDP_PKT 9u     /* u32: UDP_PKT (forwarded, proto 17)                           */
#define RTN_CNT_TCP_BYTE 10u   /* u64: TCP_BYTE                                                */
#define RTN_CNT_UDP_BYTE 12u   /* u64: UDP_BYTE                                                */

typedef struct rtn_program_info {
  uint32_t n_subscriptions;
  uint32_t n_deliver_stmts; /* packet-level callback sites in the generated code              */
  uint32_t deliver_words;   /* u64 words per statement mask (0 if no packet-level callbacks)  */
  uint32_t tree_size;       /* nodes of the collapsed PacketContinue tree                     */
  uint32_t n_conn_stmts;    /* first-packet statement sites (FilterLayer::Packet)             */
  uint32_t conn_words;      /* u64 words per first-packet statement mask                      */
  uint32_t conn_tree_size;  /* nodes of the collapsed FilterLayer::Packet tree                */
  uint32_t n_pd_stmts;      /* packet_deliver callback sites (retina_pd.h)                     */
  uint32_t n_pd_facts;      /* per-connection facts the packet_deliver filter reads            */
  uint32_t pd_tree_size;    /* nodes of the collapsed FilterLayer::PacketDeliver tree          */
} rtn_program_info_t;

/* What a first-packet statement does (the host runs it with its tracked connection data). */
#define RTN_STMT_TRACKED_PACKETS 1u /* drain tracked.packets() into a packet-level callback */
#define RTN_STMT_CALLBACK 2u        /* invoke a static/connection-level callback          */
#define RTN_STMT_STREAM 3u          /* tracked.streaming_<id>.matched()                   */

const char* rtn_last_error(void);

/* filtergen: subscription spec (TOML text, [[subscriptions]] filter/datatypes/callback) */
int32_t rtn_program_compile(const char* spec, size_t len, rtn_program_t** out);
/* Convenience: a single subscription (filter string + comma-separated datatypes + callback). */
int32_t rtn_program_compile_filter(const char* filter, const char* datatypes, const char* callback,
                                   rtn_program_t** out);
int32_t rtn_program_info(const rtn_program_t* p, rtn_program_info_t* info);
/* Text outputs: return the length needed (excluding NUL); copy at most cap-1 bytes + NUL. */
size_t rtn_program_tree(const rtn_program_t* p, char* buf, size_t cap);   /* PTree Display   */
size_t rtn_program_rust(const rtn_program_t* p, char* buf, size_t cap);   /* filtergen view   */
size_t rtn_program_source(const rtn_program_t* p, char* buf, size_t cap); /* full HIP source  */
/* Statement k of a deliver mask -> subscription index / Payload flag. */
int32_t rtn_program_deliver_table(const rtn_program_t* p, uint32_t* sub_ids, uint8_t* is_payload,
                                  uint32_t cap);
/* Statement k's callback name (the subscription's `callback`; 0 if k is out of range). */
size_t rtn_program_deliver_callback(const rtn_program_t* p, uint32_t k, char* buf, size_t cap);
/* The packet-level keep/drop filter for the NIC (FilterFactory.filter_str, get_hw_filter in
 * filtergen/src/lib.rs:233-238): the PacketContinue tree's paths joined with "or" ("" = keep all).
 * Installing it as rte_flow rules (core/src/filter/hardware) is the caller's business. */
size_t rtn_program_hw_filter(const rtn_program_t* p, char* buf, size_t cap);
/* The first-packet filter (FilterLayer::Packet): its tree, its filtergen view, and statement
 * k of a conn_dlv mask -> subscription index / RTN_STMT_* kind. */
size_t rtn_program_conn_tree(const rtn_program_t* p, char* buf, size_t cap);
size_t rtn_program_conn_rust(const rtn_program_t* p, char* buf, size_t cap);
int32_t rtn_program_conn_table(const rtn_program_t* p, uint32_t* sub_ids, uint8_t* kinds, uint32_t cap);
/* A collapsed tree as JSON (layer 0 = PacketContinue, 1 = Packet, 2 = PacketDeliver): nodes with pred, actions,
 * deliver/stream subscription ids, if_else and children -- for tooling and the test oracle. */
size_t rtn_program_tree_json(const rtn_program_t* p, uint32_t layer, char* buf, size_t cap);
/* The packet_deliver filter (retina_pd.h): JSON {"facts": [{kind: "service"|"session", pred,
 * protocol}], "stmts": [{sub, payload, callback, loops: [[node id, fact], ...]}]} in code order,
 * and its filtergen view. */
size_t rtn_program_pd_json(const rtn_program_t* p, char* buf, size_t cap);
size_t rtn_program_pd_rust(const rtn_program_t* p, char* buf, size_t cap);
/* Compile the program's kernel for gfx950 (hiprtc; needs no GPU). Returns code-object bytes. */
int32_t rtn_program_code_object(rtn_program_t* p, const uint8_t** data, size_t* len);
void rtn_program_destroy(rtn_program_t* p);

/* Load a program on `device` (compiles on first use; cached per process). */
int32_t rtn_pc_create(const char* spec, size_t len, int device, rtn_pc_t** out);
int32_t rtn_pc_create_from_program(rtn_program_t* p, int device, rtn_pc_t** out);
/* Launch on `stream` (a hipStream_t, NULL = default). Asynchronous. */
int32_t rtn_pc_run(rtn_pc_t* pc, const rtn_batch_t* in, rtn_pc_out_t* out, void* stream);
/* RTN_STATUS_* bits raised by this context's runs without counters since the last call, then
 * cleared. Waits for the context's last such run (not for the device or other streams). */
int32_t rtn_pc_take_status(rtn_pc_t* pc, uint32_t* status);
/* accepted_idx / n_accepted (the compaction form of SURVEY §8(b)) from any of the output
 * bitmaps (pc_bitmap, fwd_bitmap, dlv_bitmap), on `stream` after the run that wrote it:
 * idx[k] = the frame index of the k-th set bit among frames [0, n), in frame order (idx holds
 * up to n entries); *n_set = their count (both device memory). chunk_base (optional,
 * [ceil(n / RTN_CHUNK_FRAMES) + 1]): the number of set bits before each chunk, so the record at
 * RTN_REC_INDEX(n, c, k) belongs to frame idx[chunk_base[c] + k] (fwd_bitmap: l4, conn,
 * rtn_ct_entry_t; dlv_bitmap: the record at dlv_records[c * RTN_CHUNK_FRAMES + k]), and
 * chunk_base[last] = *n_set.
 * Asynchronous; one scratch buffer per context, so calls on one context must not overlap. */
int32_t rtn_pc_index(rtn_pc_t* pc, const uint64_t* bitmap, uint32_t n, uint32_t* idx, uint32_t* n_set,
                     uint32_t* chunk_base, void* stream);
/* Launch shape of one of the context's kernel instances (diagnostics): layout 0 = monolithic
 * slots, 1 = 64-byte slots, 2 = split, 3 = compact split; conn != 0 = the connection-stage
 * instance. waves_per_simd is the runtime's occupancy for blocks of `threads` (registers and LDS);
 * chunks_per_wave is what rtn_pc_run passes the compact split kernel (2 below 4 waves per SIMD). */
typedef struct rtn_kernel_info {
  uint32_t regs;            /* HIP_FUNC_ATTRIBUTE_NUM_REGS                 */
  uint32_t lds_bytes;       /* static LDS per block                        */
  uint32_t threads;         /* threads per block                           */
  uint32_t waves_per_simd;  /* occupancy (0 if the runtime cannot say)     */
  uint32_t chunks_per_wave;
} rtn_kernel_info_t;
int32_t rtn_pc_kernel_info(const rtn_pc_t* pc, uint32_t layout, uint32_t conn, rtn_kernel_info_t* info);
/* Workgroups per launch (0 = default). */
int32_t rtn_pc_set_grid(rtn_pc_t* pc, uint32_t blocks);
int32_t rtn_pc_destroy(rtn_pc_t* pc);

/* Bytes the caller must allocate for each output array for n frames (for deliver_words). */
size_t rtn_out_bitmap_bytes(uint32_t n);
size_t rtn_out_l4_bytes(uint32_t n);
size_t rtn_out_addr6_bytes(uint32_t n);
size_t rtn_out_dlv_bytes(uint32_t n, uint32_t deliver_words);
size_t rtn_out_conn_bytes(uint32_t n);
size_t rtn_out_conn_dlv_bytes(uint32_t n, uint32_t conn_words);
size_t rtn_out_seqack_bytes(uint32_t n);

#ifdef __cplusplus
}
#endif

#endif /* RETINA_PC_H */
