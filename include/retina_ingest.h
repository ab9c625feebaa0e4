/*
 * retina_ingest.h — offline ingest for the MI355X packet stage: a capture file -> slot slab.
 *
 * Replaces, for the batched path, what the reference's offline runtime does before the packet
 * filter (core/src/runtime/offline.rs:64-82):
 *   - Capture::from_file(pcap) (pcap crate; libpcap and pcapng files)         offline.rs:64-65
 *   - skip a frame whose original (wire) length exceeds the configured mtu    offline.rs:68-70
 *   - Mbuf::from_bytes(frame.data): mbuf data = the captured bytes, data_len = their count
 *                                                            core/src/memory/mbuf.rs:56-76
 * Frames are packed, in file order, into the slot layout rtn_pc_run reads (retina_pc.h): slot i
 * (stride bytes) receives the first min(data_len[i], stride) captured bytes; bytes past that
 * are left as they were (the kernel never reads past data_len). Same error conventions as
 * retina_pc.h (0 or a negative RTN_* code; rtn_last_error()).
 */
#ifndef RETINA_INGEST_H
#define RETINA_INGEST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rtn_pcap rtn_pcap_t;

typedef struct rtn_pcap_stats {
  uint64_t frames;       /* frames read from the file                                   */
  uint64_t skipped_mtu;  /* ... of which skipped: original length > mtu (offline.rs:68) */
  uint64_t packed;       /* ... of which handed to the filter                          */
  uint64_t bytes;        /* captured bytes of the packed frames (offline.rs nb_bytes)  */
} rtn_pcap_stats_t;

/* Open a libpcap (either byte order, us or ns timestamps) or pcapng capture. */
int32_t rtn_pcap_open(const char* path, uint32_t mtu, rtn_pcap_t** out);
/* Pack up to `cap` frames into slab/data_len (host memory, e.g. pinned); *n = frames packed,
 * 0 at end of file. A captured frame longer than 65535 bytes (beyond Mbuf::data_len's u16)
 * fails with RTN_ERANGE. */
int32_t rtn_pcap_next_batch(rtn_pcap_t* p, uint8_t* slab, uint64_t stride, uint16_t* data_len, uint32_t cap,
                            uint32_t* n);
/* The same in the compact split layout (retina_pc.h, RTN_BATCH_EXT_COMPACT): head slot k (64 B)
 * receives the first min(data_len, 64) bytes; a frame for which rtn_ext_needed() holds also gets
 * the next ext row (its bytes [64, 128)); ext_chunk[c] receives the first row of chunk c (RTN_CHUNK_FRAMES)
 * (ceil(cap / RTN_CHUNK_FRAMES) entries). *rows = rows written. The batch ends early, at a frame, when ext_cap
 * rows are used (allocate cap rows to never end early); if that frame is the batch's first, the call
 * fails with RTN_ERANGE (*n = 0), so that *n == 0 with RTN_OK always means end of file. */
int32_t rtn_pcap_next_batch_split(rtn_pcap_t* p, uint8_t* head, uint8_t* ext, uint32_t ext_cap, uint32_t* ext_chunk,
                                  uint16_t* data_len, uint32_t cap, uint32_t* n, uint32_t* rows);
/* The same frames with the capture walk on the GPU (the host copies the file's bytes, the device
 * finds the records): a window of the capture (rtn_pcap_gpu_window, default 64 MiB) is copied to
 * HBM as it is (the copy engine reads the window's pages of the file mapping, registered with
 * HIP; the next window is prefetched on an internal stream while this one's batches run; device
 * memory: two buffers of twice the window), and gfx950 kernels find its record chain in parallel (speculated per 4-KiB
 * segment, then confirmed exactly from the window's first record), apply the offline runtime's
 * rules (mtu skip, data_len = captured bytes) and pack up to slab->cap kept frames into `slab`,
 * in device memory, in the gather layout of rtn_stage_gather (retina_stage.h: head slots, ext
 * rows compact within each chunk at rows [c * RTN_CHUNK_FRAMES, ...), ext_chunk[c] =
 * c * RTN_CHUNK_FRAMES; slab->ext_cap >= rtn_stage_gather_ext_rows(slab->cap)). The packing is
 * left running on `stream` (a hipStream_t; a later call on another stream waits for it). A batch
 * also ends at the end of a window, so it can hold fewer than slab->cap frames before the end of
 * the file (size the window to about cap times the mean record to keep batches full); *n,
 * the stats and the file position are final on return. *n == 0 with RTN_OK means end of file. A kept frame longer
 * than 65535 bytes ends the batch before it with RTN_ERANGE (as rtn_pcap_next_batch); pcapng
 * sections in different byte orders are refused (RTN_EINVAL). Calls may be mixed with the host
 * readers above: they share the file position and the stats. */
struct rtn_stage_slab;
int32_t rtn_pcap_next_batch_gpu(rtn_pcap_t* p, int device, const struct rtn_stage_slab* slab, uint32_t* n,
                                void* stream);
/* Window size of rtn_pcap_next_batch_gpu in bytes (64 KiB .. 1 TiB); every record must fit in one. */
int32_t rtn_pcap_gpu_window(rtn_pcap_t* p, uint64_t bytes);
int32_t rtn_pcap_stats(const rtn_pcap_t* p, rtn_pcap_stats_t* st);
/* Start again from the first frame (stats are kept). */
int32_t rtn_pcap_rewind(rtn_pcap_t* p);
void rtn_pcap_close(rtn_pcap_t* p);

#ifdef __cplusplus
}
#endif

#endif /* RETINA_INGEST_H */
