/*
 * retina_stage.h — staging DPDK RX bursts into the batch layout rtn_pc_run reads.
 *
 * Replaces, for the batched path, the step between rx_burst and the packet filter
 * (core/src/lcore/rx_core.rs:57-73 rx_burst into a 32-mbuf array, :117-141 the per-mbuf loop):
 * the reference reads each header straight out of its mbuf at buf_addr + data_off + offset
 * (Mbuf::get_data, core/src/memory/mbuf.rs:125-141), one mbuf at a time. Here a whole set of
 * bursts is gathered, by mbuf data pointer (= buf_addr + data_off) and Mbuf::data_len
 * (mbuf.rs:95-97), into the compact split layout of retina_pc.h (RTN_BATCH_EXT_COMPACT): a 64-B
 * head slot per frame, and a 64-B ext row (bytes [64, 128)) only for the frames rtn_ext_needed()
 * names. Two forms:
 *
 *  (a) rtn_stage_mbufs: pinned host threads copy the bytes into host memory (e.g. pinned, for a
 *      host -> HBM copy); ext rows are exactly compact (ext_chunk = exclusive prefix over chunks).
 *  (b) rtn_stage_gather: a gfx950 kernel reads the mbufs straight out of a host mbuf pool the GPU
 *      maps (rtn_mbuf_pool_register = hipHostRegister), through the pointer array, and writes the
 *      layout in HBM: no host copy. Ext rows are compact within each 256-frame chunk
 *      (ext_chunk[c] = c * RTN_CHUNK_FRAMES: a chunk's needed rows are adjacent, so the filter
 *      kernel reads them as dense as in form (a)), so ext holds rtn_stage_gather_ext_rows(n) rows.
 *
 * Contract for the data pointers (both forms): data[i] must be readable for 128 bytes (true of
 * every DPDK RX mbuf: its data room is >= 2048 B past data_off). Bytes of a head slot or ext row
 * past the frame's data_len are copied from the buffer as they are; the filter never reads them
 * (every header read is bounded by data_len, mbuf.rs:125-135). The caller keeps ownership of the
 * mbufs; nothing holds their pointers after the call (form (b): after the stream has passed the
 * gather kernel). Same error conventions as retina_pc.h (0 or a negative RTN_* code,
 * rtn_last_error()).
 */
#ifndef RETINA_STAGE_H
#define RETINA_STAGE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Where a staged batch goes. Host memory for rtn_stage_mbufs, device memory for rtn_stage_gather.
 * head: [cap][64]; ext: [ext_cap][64]; ext_chunk: [ceil(cap / RTN_CHUNK_FRAMES)]; data_len: [cap].
 * head and ext must be 16-byte aligned. */
typedef struct rtn_stage_slab {
  uint8_t* head;
  uint8_t* ext;
  uint32_t* ext_chunk;
  uint16_t* data_len;
  uint32_t cap;     /* frames the slab holds        */
  uint32_t ext_cap; /* ext rows the slab holds      */
} rtn_stage_slab_t;

/* (a) Host threads. A stager owns `threads` worker threads (0 = gather on the calling thread),
 * pinned to cpus[k] when cpus is not NULL. One stager per RX thread (not thread-safe). */
typedef struct rtn_stager rtn_stager_t;
int32_t rtn_stager_create(uint32_t threads, const int32_t* cpus, rtn_stager_t** out);
void rtn_stager_destroy(rtn_stager_t* st);
/* Gather frames data[0..n) (data_len[i] bytes each, of which the first 128 matter) into slab
 * frames [0, n): head slot i = the frame's first 64 bytes, data_len[i]; the frames for which
 * rtn_ext_needed(head, data_len) holds get ext rows 0, 1, ... in frame order, and ext_chunk[c] =
 * the row of chunk c's first such frame. *rows = rows written; *dl_max = the largest data_len
 * (<= 64 means the 64-byte-slot kernel may run without ext: RTN_BATCH_DL_LE64). RTN_ERANGE if
 * n > cap or the frames need more than ext_cap rows (allocate cap rows to never fail). */
int32_t rtn_stage_mbufs(rtn_stager_t* st, const uint8_t* const* data, const uint16_t* data_len, uint32_t n,
                        const rtn_stage_slab_t* slab, uint32_t* rows, uint16_t* dl_max);

/* (b) GPU pull. Register a host memory range that holds mbuf buffers (a DPDK mempool's memory)
 * for `device`: hipHostRegister, so the GPU reads it over PCIe. The range stays registered until
 * rtn_mbuf_pool_destroy. The gather kernel only dereferences pointers p with base <= p and
 * p + 128 <= base + bytes; any other pointer gives its frame data_len 0 (nothing parses, the
 * frame is dropped) and raises RTN_STATUS_BAD_MBUF. */
typedef struct rtn_mbuf_pool rtn_mbuf_pool_t;
#define RTN_STATUS_BAD_MBUF 8u /* a data pointer outside the registered pool (not dereferenced) */
int32_t rtn_mbuf_pool_register(void* base, size_t bytes, int device, rtn_mbuf_pool_t** out);
int32_t rtn_mbuf_pool_destroy(rtn_mbuf_pool_t* pool);
/* Ext rows rtn_stage_gather writes for n frames: ceil(n / RTN_CHUNK_FRAMES) * RTN_CHUNK_FRAMES. */
uint32_t rtn_stage_gather_ext_rows(uint32_t n);
/* Launch the gather on `stream` (asynchronous): data (the n data pointers, host virtual addresses
 * into the pool) and data_len must be memory the device can read (device memory, or pinned /
 * registered host memory). Writes, in device memory: slab->head slots, slab->data_len, the ext
 * rows of each chunk c at rows [c * 256, c * 256 + its needing frames), ext_chunk[c] = c * 256.
 * Then run rtn_pc_run with RTN_BATCH_EXT_COMPACT, ext_rows = rtn_stage_gather_ext_rows(n).
 * status: optional device u32 that receives RTN_STATUS_BAD_MBUF (atomic OR); NULL = the pool's
 * sticky status word (rtn_mbuf_pool_take_status). */
int32_t rtn_stage_gather(rtn_mbuf_pool_t* pool, const uint64_t* data, const uint16_t* data_len, uint32_t n,
                         const rtn_stage_slab_t* slab, uint32_t* status, void* stream);
/* Status bits of gathers without a status pointer since the last call, then cleared (waits for
 * the pool's last such gather). */
int32_t rtn_mbuf_pool_take_status(rtn_mbuf_pool_t* pool, uint32_t* status);

#ifdef __cplusplus
}
#endif

#endif /* RETINA_STAGE_H */
