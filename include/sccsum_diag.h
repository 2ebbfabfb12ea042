/*
 * sccsum_diag.h — DIAGNOSTIC knobs of libsccsum (A/B timing, cross-checks,
 * bench's read ceiling).  Not part of the production boundary in sccsum.h:
 * nothing a caller of the checksum API needs is here.  Every knob applies to
 * launches made later by the CALLING HOST THREAD only (thread-local), so one
 * shard's experiment never changes another thread's launches.  Results never
 * depend on a knob: every setting computes the same bits.
 */
#ifndef SCCSUM_DIAG_H
#define SCCSUM_DIAG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Kernel family for this thread's later launches.
 * 0 = default: flat kernel, form 16 (>= 512 Ki packets and >= 256 MiB) else 15;
 *     variant 2 for sparse layouts (bytes_len / n >= max_len + 64).
 * 1 = one packet per wave, per-lane byte masks (an independent second
 *     implementation kept for cross-checking; in-place fill uses the flat
 *     kernel whatever the variant).
 * 2 = one packet per 16-lane row, four packets per wave at a time (sparse
 *     layouts: packets far apart, e.g. in mbuf slots).
 * 14-16 = flat kernel forms: each tile's byte extent streamed densely, unit
 *     sums prefix-scanned across the wave; U = 8 (14, 15: the next chunk in
 *     flight) or 16 (16) units per lane per chunk.  (The U = 2 / 4 forms and
 *     the rolling-row forms lost their A/Bs and were removed in round 2.)
 * SCCSUM_EINVAL for anything else. */
int sccsum_set_kernel_variant(int variant);

/* Cap the launch grid at `blocks` 256-thread workgroups per compute unit
 * (default 8).  SCCSUM_EINVAL outside 1..32. */
int sccsum_set_blocks_per_cu(int blocks);

/* Simple kernel (variant 1): force U, the 16-byte units each lane loads per
 * step (1, 2, 4 or 8; 0 = choose from max_len). */
int sccsum_set_group_units(int units);

/* Flat kernel: cap a tile (packets a wave plans at once) at 1..64 (default 64). */
int sccsum_set_tile_packets(int packets);

/* Flat kernel: target bytes per tile (default 49152; 0 = only the 64-packet cap). */
int sccsum_set_tile_bytes(int bytes);

/* Flat kernel: tiles dequeued from a counter slot of the device's pool (1, the
 * default; a launch that finds no free slot deals them round robin anyway) or
 * dealt round robin (0). */
int sccsum_set_dynamic_tiles(int on);

/* Flat kernel: cut the launch's last tiles (quarters / 4 tiles per wave of the
 * grid, 0..64) into `split` sub-tiles each (1 = no split, 2, 4 or 8), so the
 * launch's drain waits on short tiles. */
int sccsum_set_tail_split(int split, int quarters);

/* Flat kernel: cache policy of the per-tile result stores (0 = plain global
 * store; buffer stores with 1 = nt, the default, 2 = sc1, 3 = sc0 sc1,
 * 4 = sc0).  SCCSUM_EINVAL outside 0..4. */
int sccsum_set_out_policy(int policy);
/* Engine result stores: written through, sc0 sc1 (1, default), or stored as a
 * launch stores them (out_policy and the 128-byte rule) with an agent-scope
 * release before each step's completion count (0).  A/B only. */
int sccsum_set_engine_write_through(int on);
/* Engine runs started later by this thread: how long the grid may go without
 * a new step before its waiting waves give up and the run reports
 * SCCSUM_EIDLE, overriding the engine's own limit (sccsum_engine_opts.idle_ms)
 * when > 0 (1 .. 3 600 000 ms; 0, the default, = no override). */
int sccsum_set_engine_idle_ms(int ms);
/* Engine steps submitted later by this thread: every k-th step's tiles wait
 * until the step before it is done (a barrier that lines up dequeue groups
 * drifting apart over a long run).  -1 (default) = every
 * 10th step of those with at least 2 tiles per wave of the grid; 0 = never;
 * k = every k-th step.  SCCSUM_EINVAL outside -1 .. 65536. */
int sccsum_set_engine_sync_every(int steps);

/* In-place fills (SCCSUM_FILL_L4 / SCCSUM_FILL_ICMP_ECHO, launches and engine
 * fill steps) of at most `frames` frames run in one pass: the generate tiles
 * store the fields themselves (default 524 288; 0 = always two passes).
 * SCCSUM_EINVAL below 0. */
int sccsum_set_fill_single_max(int frames);

/* Flat kernel forms without a chunk in flight (U 8 form 14, U 16): a run's
 * last chunk loads and scans only the rows its units reach, U / 8 .. U (1, the
 * default), or always U rows (0).  SCCSUM_EINVAL otherwise. */
int sccsum_set_short_chunks(int on);

/* Flat kernel: each run's streamed extent starts on a boundary of `units`
 * 16-byte units (1, 4 = 64 B or 8 = 128 B, the default; clamped to the
 * batch's first unit), so a wave's 1 KiB load rows cover whole cache lines.
 * SCCSUM_EINVAL otherwise. */
int sccsum_set_run_align(int units);

/* Stream-read `bytes` (multiple of 16) from d_src with the same
 * load width as the checksum kernels and write one 64-bit word per workgroup
 * to d_sink (capacity >= sccsum_read_probe_blocks()).  Used by bench.py as
 * the measured HBM read ceiling. */
int sccsum_read_probe(const void* d_src, uint64_t bytes, uint64_t* d_sink, void* stream);
int sccsum_read_probe_blocks(void);

/* Burst queues driven from this thread: how a batch holding zero-copy packets
 * (sccsum_burst_submit_mapped) runs.  2 (default) = one launch of the
 * fragment-list kernel that reads the pinned metadata, descriptors and
 * fragments where they lie and writes the results into the pinned result
 * block (no copies); 1 = metadata H2D, fragment-list kernel, results D2H;
 * 0 = metadata H2D, sccsum_gather into the batch, sum the batch, results D2H
 * (the two-pass form).  SCCSUM_EINVAL for anything else. */
int sccsum_set_burst_fused(int on);

#ifdef __cplusplus
}
#endif

#endif /* SCCSUM_DIAG_H */
