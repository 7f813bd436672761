/*
 * clgraph.h -- C ABI of the MI355X graph engine: ONE reference Chandy-Lamport
 * simulation (sim.go ChandyLamportSim) over a large topology, state in HBM.
 *
 * Where clsnap.h batches many copies of a small scenario (one wave segment per
 * instance), cl_graph runs a single instance whose nodes and channels span the whole
 * GPU: BASELINE configs 4 (2^20-node random 8-out-regular digraph, one snapshot under
 * continuous token traffic) and 5 (100k-node power-law graph, 4,096 overlapping
 * snapshots).  It keeps the reference's semantics bit-exactly -- tick order, same-tick
 * visibility, the global delay-draw order, per-channel recording -- and runs the
 * reference's test_data scenarios too (parity-tested against the golden snapshots).
 *
 * Conventions follow clsnap.h: int return codes (CL_OK / CL_E_*), cl_last_error(),
 * caller-allocated buffers, one host thread per cl_graph, node order = getSortedKeys
 * (common.go:135-146) rank, channel c = the c-th link in (src rank, dest rank) order.
 * Per-run fatal conditions become a status (CL_INST_*) and freeze the simulation.
 *
 * Event model.  The engine executes a program of steps; step k (simulator time k) is:
 *   1. synthetic traffic sends of step k (if configured, cl_graph_set_traffic),
 *   2. host events (cl_graph_send_tokens / cl_graph_start_snapshot) in call order,
 *   3. one Tick (sim.go:71-95).
 * Host calls only append to the program; cl_graph_flush() executes what is pending
 * on the GPU, and cl_graph_rerun() replays the whole program from the initial state.
 */
#ifndef CLGRAPH_H
#define CLGRAPH_H

#include <stdint.h>

#include "clsnap.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- checksums (cl_graph_get_checksums), int64, all-reducible across ranks ---- */
#define CL_GSUM_OK 0             /* 1 if the run's status is CL_INST_OK */
#define CL_GSUM_DELIVERED 1      /* delivered packets (sim.go:85 pops) */
#define CL_GSUM_COMPLETED 2      /* globally completed snapshots */
#define CL_GSUM_CUT_RESIDUAL 3   /* sum over completed snapshots |tokens + recorded - total| */
#define CL_GSUM_FINAL_RESIDUAL 4 /* |final tokens + in-flight tokens - total| (checkTokens) */
#define CL_GSUM_DIGEST 5         /* sum of per-snapshot content digests */
#define CL_GSUM_IN_FLIGHT 6      /* token payloads still queued */
#define CL_NUM_GSUMS 7

typedef struct cl_graph cl_graph;

int cl_graph_create(cl_graph** out);
int cl_graph_destroy(cl_graph* g);
int cl_graph_set_device(cl_graph* g, int32_t device_ordinal);

/* ---- topology (before the first event) ------------------------------------- */
/* AddNode / AddLink (sim.go:40-56; node.go:45-55,87-94) and readTopologyFile
 * (test_common.go:29-68): string ids, ranked by lexicographic order at freeze. */
int cl_graph_add_node(cl_graph* g, const char* id, int64_t tokens);
int cl_graph_add_link(cl_graph* g, const char* src, const char* dest);
int cl_graph_read_topology_text(cl_graph* g, const char* text);
int cl_graph_read_topology_file(cl_graph* g, const char* path);
/* Bulk topology by rank: node r is "N" + r zero-padded to id_width digits (so rank ==
 * lexicographic order; id_width = 0 picks the digits of n_nodes-1), tokens[r]; the
 * links AddLink(src[i], dst[i]) with self links ignored and duplicates collapsed. */
int cl_graph_set_topology(cl_graph* g, int32_t n_nodes, int32_t id_width, const int64_t* tokens,
                          int64_t n_edges, const int32_t* src, const int32_t* dst);
/* Synthetic graphs:
 * regular: `degree` random permutations pi_p (Fisher-Yates driven by
 *   cl_counter_hash(seed, p, i)), links v -> pi_p(v);
 * powerlaw: `targets` links per node to ranks drawn from Zipf(exponent) over rank,
 *   plus ring links v -> v+1 and v -> v-1 when ring != 0.
 * Every node starts with `tokens` tokens. */
int cl_graph_generate_regular(cl_graph* g, int32_t n_nodes, int32_t degree, int64_t tokens, uint64_t seed);
int cl_graph_generate_powerlaw(cl_graph* g, int32_t n_nodes, int32_t targets, double exponent, int32_t ring,
                               int64_t tokens, uint64_t seed);

int cl_graph_num_nodes(cl_graph* g, int32_t* n);
int cl_graph_num_channels(cl_graph* g, int64_t* n);
/* src[c], dst[c] ranks of every channel, channel order */
int cl_graph_channels(cl_graph* g, int32_t* src, int32_t* dst);
/* node id of a rank, NUL-terminated into buf[cap] (CL_E_LIMIT if cap <= its length) */
int cl_graph_node_id(cl_graph* g, int32_t rank, char* buf, int32_t cap);
/* length of a rank's node id (bytes, without the NUL): size buf for cl_graph_node_id */
int cl_graph_node_id_length(cl_graph* g, int32_t rank, int32_t* len);

/* ---- configuration (before the first flush) -------------------------------- */
/* fifo_slots: ring slots per channel (power of two, 2..32768; deeper -> FIFO_OVERFLOW
 * status); max_snapshots: snapshot ids provisioned (0 = the program's count, at least
 * 16); max_drain_ticks bounds cl_graph_drain (HANG status). */
int cl_graph_set_limits(cl_graph* g, int32_t fifo_slots, int32_t max_snapshots, int64_t max_drain_ticks);
/* Delay source replacing rand.Intn(maxDelay) at sim.go:101; draw k of the run gets
 *   hash:     (cl_counter_hash(seed, k, 0) >> 32) % 5          (default, seed 0)
 *   go seed:  the k-th rand.Intn(5) of rand.Seed(seed)          (snapshot_test.go:20)
 *   schedule: delays[k] (values in [0, 5); DELAY_EXHAUSTED beyond n). */
int cl_graph_set_delay_hash(cl_graph* g, uint64_t seed);
int cl_graph_set_delay_go_seed(cl_graph* g, int64_t seed);
int cl_graph_set_delay_schedule(cl_graph* g, const uint8_t* delays, int64_t n);
/* Synthetic traffic: at every step k < steps, each node (rank order) holding tokens
 * with out-links sends ONE token when (uint32)cl_counter_hash(seed, k, rank) <
 * threshold, on out-link ((hash >> 32) * outdeg) >> 32 (SendTokens node.go:112-131). */
int cl_graph_set_traffic(cl_graph* g, uint64_t seed, uint32_t threshold, int64_t steps);
/* Diagnostic override of the push kernel's lanes per node: 0 = automatic (4 lanes below
 * 2^18 nodes, else 1), 1 or 4 = forced.  Results are identical either way; the tests run
 * both paths on the same graphs. */
int cl_graph_set_push_lanes(cl_graph* g, int32_t lanes);

/* ---- events ------------------------------------------------------------------ */
int cl_graph_send_tokens(cl_graph* g, const char* src, const char* dest, int64_t n);  /* sim.go:58-62 */
int cl_graph_send_tokens_rank(cl_graph* g, int32_t src, int32_t dest, int64_t n);
int cl_graph_start_snapshot(cl_graph* g, const char* node, int32_t* out_sid);         /* sim.go:105 */
int cl_graph_start_snapshot_rank(cl_graph* g, int32_t node, int32_t* out_sid);
int cl_graph_tick(cl_graph* g, int32_t n);                                             /* sim.go:71 */
/* test_common.go:123-137: tick until every snapshot started before this call has
 * completed, then maxDelay+1 more ticks.  Host-driven (checks completion between
 * ticks).  If it exceeds max_drain_ticks the run gets CL_INST_HANG and freezes: later
 * program ops do not execute. */
int cl_graph_drain(cl_graph* g);
int cl_graph_read_events_text(cl_graph* g, const char* text, int32_t* n_snapshots); /* test_common.go:79-140 */
int cl_graph_read_events_file(cl_graph* g, const char* path, int32_t* n_snapshots);

/* ---- execution ---------------------------------------------------------------- */
int cl_graph_flush(cl_graph* g);
/* Reset to the initial topology state and replay the whole program, asynchronously
 * when it has no drain (the benchmark step); cl_graph_synchronize() waits. */
int cl_graph_rerun(cl_graph* g);
int cl_graph_synchronize(cl_graph* g);
/* Device time of the runs since the previous call (HIP events on the engine stream
 * around each flush / rerun), the number of runs, and the ticks they executed. */
int cl_graph_run_time(cl_graph* g, double* total_ms, int64_t* runs, int64_t* ticks);
/* Test/benchmark aid: overwrite the run's result planes (node tokens, snapshot token maps
 * and cursors, completion ticks, counters) with 0xA5 bytes on the engine's stream, so
 * results read after the next cl_graph_rerun come from that run alone. */
int cl_graph_debug_poison_outputs(cl_graph* g);
/* Phases of the latest run: ms[0] / ticks[0] from its start to its first drain (the event
 * program's ticks: the traffic window of the synthetic workloads), ms[1] / ticks[1] the
 * drains (test_common.go:123-137); ms[1] = ticks[1] = 0 without a drain.  HIP events on the
 * engine's stream. */
int cl_graph_phase_time(cl_graph* g, double* ms /* [2] */, int64_t* ticks /* [2] */);
int cl_graph_device_bytes(cl_graph* g, int64_t* bytes);

/* ---- results (flush pending events first) ----------------------------------- */
int cl_graph_get_status(cl_graph* g, int32_t* status);
int cl_graph_get_time(cl_graph* g, int64_t* time);
int cl_graph_num_snapshots(cl_graph* g, int32_t* n);
int cl_graph_node_tokens(cl_graph* g, int64_t* out /* [num_nodes] */);
int cl_graph_snapshot_tick(cl_graph* g, int32_t sid, int32_t* tick);
/* CollectSnapshot (sim.go:134-173): tokens[rank] = tokenMap; the messages recorded on
 * channel c are msg_tokens[msg_offsets[c] .. msg_offsets[c+1]) in delivery order.
 * CL_E_NOT_COMPLETE if sid has not completed; CL_E_LIMIT (offsets written) if msg_cap
 * is too small. */
int cl_graph_collect_snapshot(cl_graph* g, int32_t sid, int64_t* tokens, int64_t* msg_offsets,
                              int64_t* msg_tokens, int64_t msg_cap);
/* CL_CNT_* counters (clsnap.h) of the run; recorded copies include channels still
 * recording at the end. */
int cl_graph_get_counters(cl_graph* g, int64_t* out /* [CL_NUM_COUNTERS] */);
int cl_graph_get_checksums(cl_graph* g, int64_t* out /* [CL_NUM_GSUMS] */);

/* ---- device event trace: the reference's debug Logger (logger.go:12-76) ---------- */
/* Record up to `capacity` LogEvents from the next run on (0 = off, the default); the next
 * flush replays the program with tracing.  A debugging aid: records go through one device
 * counter, so keep it to graphs and runs of modest size. */
int cl_graph_trace_enable(cl_graph* g, int32_t capacity);
/* The Logger's records (cl_log_event, clsnap.h) in its order -- per epoch (simulator time),
 * the tick's deliveries in sender rank order with the broadcasts and EndSnapshot records
 * they cause, then that step's traffic sends in node order, then the host events -- with
 * LogEvent.nodeTokens.  *n_events = total; CL_E_LIMIT if the run overflowed the capacity. */
int cl_graph_trace_read(cl_graph* g, cl_log_event* out, int32_t cap, int32_t* n_events);

/* ---- graph-partitioned mode --------------------------
 * ONE simulation whose nodes are split into contiguous rank ranges over several devices
 * (one process per GPU).  Each device holds the graph-sized arrays but owns the tokens,
 * out-channel FIFOs and local snapshots of its nodes [node_lo, node_hi).  There is no
 * reference interface for this (the reference is one process); the caller moves the rows
 * between devices (graph.py PartitionedGraphSim over torch.distributed all-to-all).  One
 * tick:
 *   part_pick     time++, every owned sender pops its first due head (sim.go:71-95);
 *                 returns the deliveries to other devices' receivers, rows (s, v, k, pay).
 *   part_receive  applies the deliveries addressed here (every device's rows for its
 *                 nodes, any order), handles the markers (node.go:149-171); returns the
 *                 broadcast triggers of other devices' senders, rows (s0, outdeg).
 *   part_tally    applies the reports addressed here, tallies triggers and next-step sends
 *                 of the owned senders; totals[0..2] = (trigger draws, send draws, this
 *                 device's run status).  A device that froze (engine limit) tallies
 *                 nothing, so the caller allgathers the status with the totals and, when
 *                 any device has one, freezes every device (part_freeze) before part_bases:
 *                 no device then draws from stale totals.
 *   part_bases    bases[4] = (trigger draws of lower devices, of all, send draws of lower
 *                 devices, of all); returns the first draw of each reported sender s0.
 *   part_push     replies (s0, draw0) for broadcasts triggered by other devices' senders;
 *                 pushes broadcasts and traffic sends of step `step` (queue.go:18-20).
 * The step-0 traffic is part_tally(0) + part_bases + part_push(0) with no rows.
 * part_snapshot(node) must be called on every device (each counts the draws).  Queries
 * (node tokens, counters, snapshot ticks, collect) return this device's part: its nodes,
 * the channels into them, completion over its nodes; the program calls (tick, send,
 * flush of a program) return CL_E_STATE once the partitioned run began. */
int cl_graph_part_begin(cl_graph* g, int32_t node_lo, int32_t node_hi);
int cl_graph_part_snapshot(cl_graph* g, int32_t node, int32_t* out_sid);
int cl_graph_part_pick(cl_graph* g, int32_t* rows, int64_t cap, int64_t* n_rows);
int cl_graph_part_receive(cl_graph* g, const int32_t* rows, int64_t n, int32_t* reports, int64_t cap,
                          int64_t* n_reports);
int cl_graph_part_tally(cl_graph* g, int32_t step, const int32_t* reports, int64_t n, int64_t* totals);
int cl_graph_part_bases(cl_graph* g, const int64_t* bases, const int32_t* s0, int64_t n, int64_t* draw0);
int cl_graph_part_push(cl_graph* g, int32_t step, const int64_t* replies, int64_t n);
/* Freeze this device's part of the run with `status` (no-op if it is already frozen):
 * another device froze, and the partitioned run stops everywhere at the same step. */
int cl_graph_part_freeze(cl_graph* g, int32_t status);

/* ---- partitioned mode, device-resident exchange ---------------------------------------
 * The same tick with every exchanged row kept in device memory: the caller binds four
 * device buffers it owns (torch tensors) and runs the collectives between the steps on
 * the engine's stream (cl_graph_set_stream: torch's current stream), so a tick needs no
 * host round trip (RCCL all-to-all / all-gather over xGMI with one process per GPU).
 *   send, recv  world * (cap + 1) rows of 16 B each: bucket q = a header row {rows, 0, 0, 0},
 *               then up to `cap` rows; send bucket q goes to rank q and recv bucket q came
 *               from rank q (all_to_all_single with equal splits);
 *   tot_send    4 int64 (this rank's trigger draws, send draws, status, 0);
 *   tot_recv    world * 4 int64 (all_gather of tot_send).
 * `cap` must bound every bucket: for ranks r != q, the number of r's nodes with a channel
 * into q's nodes (graph.py computes it from the topology); `span` = nodes per rank
 * (owner(v) = v / span, the block-aligned ranges of part_begin).  One tick:
 *   dev_pick      time++, pops; deliveries to other ranks' receivers -> send       [all-to-all]
 *   dev_receive   recv deliveries + own markers; broadcast reports (s0, outdeg) -> send
 *                                                                                  [all-to-all]
 *   dev_tally     recv reports, tally of triggers and next-step sends -> tot_send  [all-gather]
 *   dev_bases     draw bases from tot_recv (a frozen rank freezes every rank); replies
 *                 (s0, first draw) to the reporters -> send                       [all-to-all]
 *   dev_push      recv replies; pushes of broadcasts and the traffic of `step`.
 * The step-0 traffic: dev_seal (empty reports) [all-to-all] dev_tally(0) [all-gather]
 * dev_bases [all-to-all] dev_push(0).  The results are part_* queries as above. */
int cl_graph_part_dev_bind(cl_graph* g, int32_t world, int32_t rank, int32_t span, int64_t cap, void* send,
                           void* recv, void* tot_send, void* tot_recv);
int cl_graph_part_dev_seal(cl_graph* g);
int cl_graph_part_dev_pick(cl_graph* g);
int cl_graph_part_dev_receive(cl_graph* g);
int cl_graph_part_dev_tally(cl_graph* g, int32_t step);
int cl_graph_part_dev_bases(cl_graph* g);
int cl_graph_part_dev_push(cl_graph* g, int32_t step);
/* Run every later launch and copy of this engine on `stream` (a hipStream_t of the engine's
 * device, e.g. torch.cuda.current_stream().cuda_stream; NULL = the engine's own stream).
 * The engine waits for its own stream first. */
int cl_graph_set_stream(cl_graph* g, void* stream);

/* ---- counter hash of the synthetic workloads ------------------------------------ */
uint64_t cl_counter_hash(uint64_t seed, uint64_t a, uint64_t b);

#ifdef __cplusplus
}
#endif
#endif /* CLGRAPH_H */
