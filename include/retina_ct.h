/*
 * retina_ct.h — C ABI of the MI355X connection lookup (the table step of Retina's ConnTracker).
 *
 * Replaces, per batch, the per-packet table access of ConnTracker::process
 * (core/src/conntrack/mod.rs:80-169): `self.table.raw_entry_mut().from_key(&ConnId::new(..))`
 * on a hashlink LinkedHashMap, the Vacant-branch admission rules (Conn::new_tcp opens only on SYN
 * without ACK/RST, Conn::new_udp on any UDP frame, conntrack/conn/mod.rs:53-96; a TCP connection
 * whose first-packet filter drops is not inserted, mod.rs:139-141; size < max_connections,
 * mod.rs:127) and the resulting Occupied/Vacant outcome of every forwarded frame in frame order.
 *
 * The table lives in HBM across batches and is keyed by the canonical ConnId
 * (conntrack/conn_id.rs:115-117). A slot index is a stable connection handle: the host keeps its
 * per-connection state (Conn<T>: reassembly, parsers, tracked data) in an array indexed by slot.
 * What stays on the host: everything that depends on the session parsers or timers -- an
 * established connection that the host later removes (terminated, timed out, or dropped by the
 * protocol/session filter) is reported back with rtn_ct_remove. Within one batch the GPU assumes
 * an existing connection stays (the host, processing the batch in order, sees its own removals
 * and applies the creation rule to the following frames with the rtn_conn_t creates bit and
 * first-packet actions, reusing the same slot).
 *
 * Inputs are the outputs of rtn_pc_run for the batch, with rtn_pc_out_t.conn computed.
 * Conventions as retina_pc.h (0 / negative errno-style codes, rtn_last_error()).
 */
#ifndef RETINA_CT_H
#define RETINA_CT_H

#include <stddef.h>
#include <stdint.h>

#include "retina_pc.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rtn_ct rtn_ct_t;

/* Outcome of a forwarded frame (rtn_ct_entry_t.status & 0xff). */
#define RTN_CT_HIT 1u         /* Occupied: the connection exists when the frame arrives          */
#define RTN_CT_NEW 2u         /* Vacant, and this frame opens the connection (inserted)         */
#define RTN_CT_MISS 3u        /* Vacant, and the frame cannot open one: dropped (mid-connection) */
#define RTN_CT_NEW_DROPPED 4u /* Vacant, opener, but its first-packet filter drops it (TCP)       */
#define RTN_CT_FULL 5u        /* Vacant, opener, but the table is full ("Table full. Dropping")  */
#define RTN_CT_COLLISION 6u   /* 64-bit key fingerprint collision: resolve this frame on the host */
#define RTN_CT_PRIOR 0x100u   /* flag: the connection existed before this batch                   */
#define RTN_CT_NO_SLOT 0xFFFFFFFFu

/* Per forwarded frame, indexed like rtn_pc_out_t.l4 (RTN_REC_INDEX in retina_pc.h). */
typedef struct rtn_ct_entry {
  uint32_t slot;   /* connection handle, or RTN_CT_NO_SLOT */
  uint32_t status; /* RTN_CT_* | RTN_CT_PRIOR              */
} rtn_ct_entry_t;

typedef struct rtn_ct_stats {
  uint32_t capacity;
  uint32_t live;   /* slots holding a connection        */
  uint32_t epoch;  /* batches processed                  */
  uint32_t max_connections;
} rtn_ct_stats_t;

/* A table of 2^capacity_log2 64-byte slots on `device`, admitting at most max_connections
 * (ConnTrackConfig::max_connections). Keep the load factor below ~0.5 for short probe chains.
 * When a batch fills the table, which openers get the last slots is not frame-ordered, and
 * duplicate openers racing for one key can hold a reservation briefly, so such a batch may
 * admit a few fewer than max_connections. */
int32_t rtn_ct_create(int device, uint32_t capacity_log2, uint32_t max_connections, rtn_ct_t** out);
int32_t rtn_ct_destroy(rtn_ct_t* ct);
/* One batch (n frames, the same batch rtn_pc_run processed into `pc`): two launches on `stream`.
 * out: device array of rtn_out_ct_bytes(n) bytes, indexed like the records. */
int32_t rtn_ct_process(rtn_ct_t* ct, const rtn_pc_out_t* pc, uint32_t n, rtn_ct_entry_t* out, void* stream);
/* Remove connections (device array of slot handles); their slots become tombstones, except that a
   run of tombstones followed by an empty slot becomes empty again (it ends no probe chain). A slot
   listed twice is removed once. */
int32_t rtn_ct_remove(rtn_ct_t* ct, const uint32_t* slots, uint32_t n, void* stream);
/* Compact tombstones away: every live connection moves; new_slot (device, capacity entries)
 * receives old slot -> new slot (RTN_CT_NO_SLOT for dead ones). Synchronous. */
int32_t rtn_ct_rebuild(rtn_ct_t* ct, uint32_t* new_slot, void* stream);
int32_t rtn_ct_stats(rtn_ct_t* ct, rtn_ct_stats_t* st); /* synchronises the table's stream use */
/* Device pointer to the table (capacity * 64 bytes, layout in retina_amd/csrc/kernels/ct_kernel.hip). */
void* rtn_ct_table(rtn_ct_t* ct);
size_t rtn_out_ct_bytes(uint32_t n);

#ifdef __cplusplus
}
#endif

#endif /* RETINA_CT_H */
