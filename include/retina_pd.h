/*
 * retina_pd.h — C ABI of the MI355X PacketDeliver filter: the generated `packet_deliver`
 * (filtergen/src/lib.rs:299-304, 357-362; gen_deliver_filter, filtergen/src/deliver_filter.rs:9-151)
 * that ConnInfo::update_sdata runs on every packet of a connection holding the PacketDeliver
 * action (core/src/conntrack/conn/conn_info.rs:70-75), through Subscription::deliver_packet
 * (core/src/subscription/mod.rs:150-155). It delivers packet-level subscriptions (ZcFrame,
 * Payload, datatypes/src/packet.rs) whose filters matched at the protocol or session layer.
 *
 * One launch evaluates it for every forwarded frame of a batch, after rtn_pc_run (with addr6)
 * and rtn_ct_process. The tree tests three kinds of condition:
 *   - packet predicates (ipv4/ipv6/tcp/udp and their addr/port fields: the only packet fields a
 *     tree after PacketContinue may hold, core/src/filter/ptree.rs:406-415), evaluated on the
 *     frame's own L4Context;
 *   - service tests `matches!(conn.service(), ConnParser::X)` (filtergen/src/utils.rs:459-486);
 *   - session predicates looped over `tracked.sessions()` (deliver_filter.rs:123-151).
 * The last two depend on the connection only. The host keeps them per connection slot in
 * `state`: [slots][1 + n_pd_facts] u32 = {flags, fact 0, fact 1, ...} where flags bit 0 is
 * RTN_PD_ACTIVE (actions.packet_deliver()), a service fact is 1 if the connection's service is
 * that protocol, and a session fact is the number of the connection's tracked sessions that
 * satisfy that predicate (rtn_program_pd_json lists the facts, one per distinct predicate).
 *
 * A frame takes part if its connection existed before the batch (status RTN_CT_HIT |
 * RTN_CT_PRIOR) and its slot's flags hold RTN_PD_ACTIVE. Its output is, per statement of the
 * generated code (rtn_program_pd_json "stmts", code order), how many times that callback runs
 * for the frame: 0/1 outside session loops, the product of the enclosing loops' facts inside.
 * The reference runs the callbacks of one loop body session by session; the "loops" of each
 * statement give the host that interleaving. A connection whose state the host changes inside
 * the batch (its protocol is identified, a session is parsed, it is removed) has its later frames
 * re-evaluated by the host, as with rtn_ct_remove.
 */
#ifndef RETINA_PD_H
#define RETINA_PD_H

#include <stddef.h>
#include <stdint.h>

#include "retina_ct.h"
#include "retina_pc.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RTN_PD_ACTIVE 1u /* state flags: the connection's actions hold PacketDeliver */

/* Evaluate packet_deliver for the batch: `out` (with addr6 and conn) and `ct` as produced for the same n frames,
 * `data_len` the batch's (Payload needs the frame length), `state` [state_slots][1 + n_pd_facts]
 * in device memory. Writes pd_bitmap [ceil(n/64)] (frame has >= 1 delivery) and, for those
 * frames only, counts[record][n_pd_stmts] at the frame's record index (like l4 and ct). A
 * program without packet-level subscriptions only clears pd_bitmap. Asynchronous on `stream`. */
int32_t rtn_pd_run(rtn_pc_t* pc, const rtn_pc_out_t* out, const rtn_ct_entry_t* ct, const uint16_t* data_len,
                   uint32_t n, const uint32_t* state, uint32_t state_slots, uint32_t* counts, uint64_t* pd_bitmap,
                   void* stream);
size_t rtn_out_pd_counts_bytes(uint32_t n, uint32_t n_pd_stmts);

/* The callback sequence (statement indices, in the order the generated packet_deliver runs them)
 * of one delivering frame, from its counts row and its connection's facts: statements inside one
 * session loop run together once per matching session. *n = the sequence length; RTN_ERANGE
 * (with *n set) if it exceeds cap. */
int32_t rtn_program_pd_replay(const rtn_program_t* p, const uint32_t* counts, const uint32_t* facts, uint32_t* out,
                              uint32_t cap, uint32_t* n);

#ifdef __cplusplus
}
#endif

#endif /* RETINA_PD_H */
