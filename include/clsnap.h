/*
 * clsnap.h -- C ABI of the MI355X Chandy-Lamport batch engine.
 *
 * One cl_sim is a batch of n_instances independent copies of the reference simulator
 * (sim.go ChandyLamportSim).  Every instance shares the topology and receives the same
 * event stream (send / snapshot / tick), but draws its own per-message delays, so each
 * instance is the reference run under its own delay stream.  Instances run as
 * tick-synchronous simulations on one gfx950 GPU; results are bit-exact per instance.
 *
 * Each entry point below names the reference interface it replaces
 * (paths relative to /root/reference/chandy_lamport).  The reference is a Go package
 * with no FFI; INTEGRATION.md shows the cgo binding that maps this ABI back onto the
 * reference's Simulator API so the .top/.events drivers and snapshot_test.go run
 * unchanged.
 *
 * Conventions
 *   - Every call returns int: CL_OK (0) or a negative CL_E_* code; cl_last_error()
 *     describes the most recent failure on the calling thread.
 *   - All buffers are caller-allocated; no pointer returned by the library is owned by
 *     the caller except where stated.
 *   - One host thread drives a cl_sim (events, ticks, flush).  Event calls only append
 *     to the sim's event program; cl_flush() (or any result query) executes pending
 *     events on the GPU.  Every call holds the sim's lock, so other threads may call
 *     cl_poll_snapshot / cl_wait_snapshot / cl_collect_snapshot* concurrently -- the
 *     reference collects each snapshot on its own goroutine while the driver ticks
 *     (test_common.go:106-108, sim.go:134-173).  Those calls execute events already
 *     issued but never add a tick.
 *   - Node order everywhere is the reference's getSortedKeys order (common.go:135-146):
 *     lexicographic byte order of the node IDs ("rank").  Channel c is the c-th link in
 *     (src rank, dest rank) order -- the order Tick scans senders and out-links
 *     (sim.go:76-78).
 *   - Where the reference calls log.Fatal* on a per-run condition, the affected
 *     instance gets a CL_INST_* status and freezes; API misuse that the reference
 *     turns into a process exit or nil dereference returns a CL_E_* code instead.
 */
#ifndef CLSNAP_H
#define CLSNAP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- return codes ------------------------------------------------------- */
#define CL_OK 0
#define CL_E_INVALID (-1)        /* bad argument or handle */
#define CL_E_UNKNOWN_NODE (-2)   /* sim.go:49-54 log.Fatalf; nil *Node at sim.go:61,106 */
#define CL_E_DUPLICATE_NODE (-3) /* sim.go:42 would silently replace a wired node */
#define CL_E_PARSE (-4)          /* test_common.go parse fatals (:45,52,58,93,119,...) */
#define CL_E_IO (-5)             /* ioutil.ReadFile failure (test_common.go:30,80) */
#define CL_E_DEVICE (-6)         /* HIP error or no gfx950 device */
#define CL_E_LIMIT (-7)          /* engine limit (nodes, snapshots, token range) */
#define CL_E_STATE (-8)          /* topology change after events started, etc. */
#define CL_E_NOT_COMPLETE (-9)   /* collect of a snapshot that has not completed */

/* ---- per-instance status (cl_get_status) -------------------------------- */
#define CL_INST_OK 0
#define CL_INST_FATAL_INSUFFICIENT_TOKENS 1 /* node.go:113-116 */
#define CL_INST_FATAL_UNKNOWN_DEST 2        /* node.go:121-124 */
#define CL_INST_FIFO_OVERFLOW 3             /* engine: channel deeper than 255 packets */
#define CL_INST_HANG 4                      /* drain exceeded max ticks (test_common.go:124-132 loops forever) */
#define CL_INST_DELAY_EXHAUSTED 5           /* replayed delay schedule too short */
#define CL_INST_HIST_OVERFLOW 6             /* graph engine: token history slots exhausted */
#define CL_INST_XCHG_OVERFLOW 7             /* partitioned graph run: a device exchange bucket overflowed */

/* ---- counters (cl_get_counters), summed over instances ------------------ */
#define CL_CNT_PUSH 0      /* Queue.Push (queue.go:18) == delay draws (sim.go:101) */
#define CL_CNT_PEEK 1      /* Queue.Peek inside Tick (sim.go:83) */
#define CL_CNT_POP_TOKEN 2 /* delivered token packets (sim.go:85) */
#define CL_CNT_POP_MARKER 3
#define CL_CNT_RECORDED 4  /* recorded message copies (node.go:179-183) */
#define CL_CNT_COMPLETED 5 /* globally completed snapshots (sim.go:126-131) */
#define CL_CNT_INSTANCES 6 /* instances counted */
#define CL_CNT_TICKS 7     /* sum of per-instance simulator time */
#define CL_NUM_COUNTERS 8

/* ---- checksums (cl_get_checksums): int64 sums, all-reducible across ranks -- */
#define CL_SUM_INSTANCES 0       /* instances in the batch */
#define CL_SUM_OK 1              /* status OK */
#define CL_SUM_FATAL 2           /* FATAL_* statuses */
#define CL_SUM_OTHER 3           /* FIFO_OVERFLOW / HANG / DELAY_EXHAUSTED */
#define CL_SUM_DELIVERED 4       /* packets delivered by OK instances */
#define CL_SUM_SNAPSHOT_HASH 5   /* sum of snapshot content hashes over OK instances */
#define CL_SUM_CUT_RESIDUAL 6    /* sum |snapshot tokens + recorded - total| (0 = consistent cuts) */
#define CL_SUM_FINAL_RESIDUAL 7  /* sum |final tokens + in-flight tokens - total| (checkTokens) */
#define CL_SUM_COMPLETED 8       /* completed snapshots over OK instances */
#define CL_SUM_IN_FLIGHT 9       /* token packets still queued at the end (OK instances) */
#define CL_NUM_SUMS 10

typedef struct cl_sim cl_sim;

/* NewSimulator (sim.go:28-37) for n_instances independent instances. No GPU work. */
int cl_sim_create(int64_t n_instances, cl_sim** out);
/* Wakes every thread blocked in cl_wait_snapshot (they return CL_E_STATE) and waits for
 * them to leave before freeing the sim; no other call may overlap it. */
int cl_sim_destroy(cl_sim* sim);

/* AddNode (sim.go:40-43; node.go:45-55). Token counts must fit int32 in total. */
int cl_add_node(cl_sim* sim, const char* id, int64_t tokens);
/* AddLink (sim.go:46-56; node.go:87-94): self links ignored, duplicates replace. */
int cl_add_link(cl_sim* sim, const char* src, const char* dest);
/* readTopologyFile (test_common.go:29-68) on a file path / on text. */
int cl_read_topology_file(cl_sim* sim, const char* path);
int cl_read_topology_text(cl_sim* sim, const char* text);

/* Engine configuration (before the first flush). */
int cl_set_device(cl_sim* sim, int32_t device_ordinal);
/* fifo_lds_slots: per-channel packets kept in LDS (power of two, 2..64; deeper
 * channels spill to HBM), or 0 to size it automatically for occupancy (default).
 * max_drain_ticks bounds the drain loop (HANG status). */
int cl_set_limits(cl_sim* sim, int32_t fifo_lds_slots, int64_t max_drain_ticks);

/* Delay source replacing rand.Intn(maxDelay) at sim.go:101.
 * Go stream: instance i draws from rand.Seed(seed_base + i) -- the reference's own
 * generator (snapshot_test.go:20), restated bit-exactly and precomputed on the host. */
int cl_set_delay_go_seeds(cl_sim* sim, int64_t seed_base);
/* Explicit schedule: delays[i * draws_per_instance + k] in [0, 5) is the k-th draw
 * of instance i.  Copied; the caller may free it after the call. */
int cl_set_delay_schedule(cl_sim* sim, const uint8_t* delays, int64_t draws_per_instance);

/* ProcessEvent(PassTokenEvent) -> SendTokens (sim.go:58-62; node.go:112-131). */
int cl_send_tokens(cl_sim* sim, const char* src, const char* dest, int64_t n);
/* ProcessEvent(SnapshotEvent) -> StartSnapshot (sim.go:63-64,105-123). */
int cl_start_snapshot(cl_sim* sim, const char* node, int32_t* out_sid);
/* Tick (sim.go:71-95), n times. */
int cl_tick(cl_sim* sim, int32_t n);
/* The drain of readEventsFile (test_common.go:123-137): tick until every started
 * snapshot has completed in an instance, then maxDelay+1 more ticks (per instance). */
int cl_drain(cl_sim* sim);
/* readEventsFile (test_common.go:79-140) incl. the drain; n_snapshots may be NULL. */
int cl_read_events_file(cl_sim* sim, const char* path, int32_t* n_snapshots);
int cl_read_events_text(cl_sim* sim, const char* text, int32_t* n_snapshots);

/* Execute pending events on the GPU and wait. */
int cl_flush(cl_sim* sim);
/* Re-run the whole event program from the initial topology state (asynchronous on
 * the sim's stream; inputs stay resident in HBM).  cl_synchronize() waits.  A replay split
 * over two streams (cl_replay_split) leaves its spill-capable half running when the call
 * returns: back-to-back cl_rerun calls overlap that half with the next replay's spill-free
 * half (they touch disjoint instances); every other call waits for it first. */
int cl_rerun(cl_sim* sim);
int cl_synchronize(cl_sim* sim);
/* Device time of the most recent cl_flush/cl_rerun kernel, from HIP events recorded by the
 * kernel dispatches themselves; a split replay's time is the longer of its two concurrent
 * halves, each timed by its own dispatch's events. */
int cl_last_kernel_ms(cl_sim* sim, double* ms);
/* Sum of exec-kernel device times (as cl_last_kernel_ms, every launch) since the previous
 * call, and the number of launches; resets the accumulator. */
int cl_kernel_time(cl_sim* sim, double* total_ms, int64_t* launches);
/* 1 in *on when the next cl_rerun runs wholly on the spill-free kernel: the layout has no HBM
 * spill rings, or the first full run of the same program with the same delays and layout
 * spilled nothing (engine-internal specialization; results are the same either way). */
int cl_replay_spill_free(cl_sim* sim, int32_t* on);
/* The replay plan of the current program (from its first full run): instances whose queues
 * outgrew the LDS rings (-1: no plan yet), and the slot from which replays run on the
 * spill-capable kernel while the slots before it run spill-free, concurrently (0: no split).
 * Engine-internal; results are the same either way. */
int cl_replay_split(cl_sim* sim, int64_t* spill_instances, int64_t* split_slot);
/* 1 in *on when the next cl_rerun launches through the replay plan's slot map (instances
 * grouped by the final tick of an earlier full run of the same program and delays, so the
 * instances sharing a wave finish together, and those that spilled last; engine-internal,
 * results unchanged). */
int cl_replay_mapped(cl_sim* sim, int32_t* on);

/* Which exec kernel runs the program (engine-internal; results are identical):
 *   CL_ENGINE_AUTO   the instance-per-lane kernel, compiled at run time for this topology
 *                    (hipRTC), wherever the topology fits it (<= 16 nodes, every degree <= 4,
 *                    <= 16 snapshot ids); else -- or when run-time compilation fails -- the
 *                    node-parallel kernel
 *   CL_ENGINE_NODES  the node-parallel kernel (one lane per node)
 *   CL_ENGINE_LANES  the instance-per-lane kernel; CL_E_LIMIT where the topology does not fit
 * cl_exec_engine reports the kernel the most recent launch used (0 before any). */
#define CL_ENGINE_AUTO 0
#define CL_ENGINE_NODES 1
#define CL_ENGINE_LANES 2
int cl_set_exec_engine(cl_sim* sim, int32_t engine);
int cl_exec_engine(cl_sim* sim, int32_t* engine);
/* Run-time kernel compilations of this process so far and their total wall time. */
int cl_jit_stats(double* compile_ms, int64_t* compiles);
/* Compile the instance-per-lane kernels for this sim's topology and layout without loading
 * them (no device needed): CL_OK, or CL_E_LIMIT (the topology does not fit them) / CL_E_DEVICE
 * (compilation failed); the compiler log goes to log (log_cap bytes, may be NULL). */
int cl_lanes_compile_check(cl_sim* sim, double* compile_ms, char* log, int64_t log_cap);

/* Test/benchmark aid (no reference counterpart): overwrite every result plane the exec
 * kernel writes -- node snapshot records, completion ticks, per-instance result rows,
 * final node tokens -- with the byte 0xA5 on the sim's stream, so that results read after
 * the next cl_rerun can only come from that launch.  No-op before the first execution. */
int cl_debug_poison_outputs(cl_sim* sim);

/* ---- topology queries (host only) ---------------------------------------- */
int cl_num_nodes(const cl_sim* sim, int32_t* n);
int cl_node_id(const cl_sim* sim, int32_t rank, const char** id); /* owned by sim */
int cl_num_channels(const cl_sim* sim, int32_t* n);
int cl_channel(const cl_sim* sim, int32_t ch, int32_t* src_rank, int32_t* dest_rank);
int cl_num_snapshots(const cl_sim* sim, int32_t* n);
int cl_num_instances(const cl_sim* sim, int64_t* n);
/* Delay draws per instance the current event program can consume (upper bound). */
int cl_delay_draws_needed(const cl_sim* sim, int64_t* draws);
/* Bytes of GPU memory the batch holds (after flush). */
int cl_device_bytes(const cl_sim* sim, int64_t* bytes);

/* ---- results (flush pending events first) -------------------------------- */
int cl_get_status(cl_sim* sim, int32_t* out /* [n_instances] */);
int cl_get_time(cl_sim* sim, int32_t* out /* [n_instances] */);
/* Final node tokens (checkTokens, test_common.go:298-302), rank order. */
int cl_node_tokens(cl_sim* sim, int64_t inst, int64_t* out /* [num_nodes] */);
/* Completion tick of snapshot sid in instance inst, -1 if not complete. */
int cl_snapshot_tick(cl_sim* sim, int32_t sid, int64_t inst, int32_t* tick);
/* CollectSnapshot (sim.go:134-173) of one instance: tokens[rank] = tokenMap, and the
 * recorded messages as a CSR over channels: messages of channel c are
 * msg_tokens[msg_offsets[c] .. msg_offsets[c+1]) in delivery order.  Returns
 * CL_E_NOT_COMPLETE if the snapshot has not completed in that instance; if msg_cap is
 * too small, offsets are still written and CL_E_LIMIT is returned. */
int cl_collect_snapshot(cl_sim* sim, int32_t sid, int64_t inst, int64_t* tokens,
                        int64_t* msg_offsets /* [num_channels + 1] */, int64_t* msg_tokens,
                        int64_t msg_cap);
/* Completion of snapshot sid over instances [inst_lo, inst_hi) -- the global
 * WaitGroup of sim.go:116-117,126-131 per instance: *n_complete = instances whose
 * snapshot has completed after every event issued so far (pending events are executed,
 * no tick is added).  Non-blocking apart from that execution. */
int cl_poll_snapshot(cl_sim* sim, int32_t sid, int64_t inst_lo, int64_t inst_hi, int64_t* n_complete);
/* The blocking side of CollectSnapshot (sim.go:137-140): wait until snapshot sid has
 * completed in every instance of [inst_lo, inst_hi).  The caller is a collector thread;
 * it is woken after each execution of the driver's events (cl_flush, queries) and after
 * every cl_tick / cl_drain, and re-checks (executing the pending events itself, so a
 * driver that only calls Tick() -- the reference's pattern -- completes the wait).  timeout_ms < 0 waits forever; on timeout returns CL_E_NOT_COMPLETE with
 * *n_complete (may be NULL) set.  It also returns CL_E_NOT_COMPLETE at once when every
 * instance of the range has either completed or stopped with a non-OK status (the
 * reference process would have exited at that log.Fatal; such an instance never
 * completes).  Never ticks. */
int cl_wait_snapshot(cl_sim* sim, int32_t sid, int64_t inst_lo, int64_t inst_hi, int64_t timeout_ms,
                     int64_t* n_complete);
/* CollectSnapshot (sim.go:134-173) of instances [inst_lo, inst_hi) at once:
 * tokens[(i - inst_lo) * N + rank] (-1 for an instance whose snapshot has not
 * completed, with complete[i - inst_lo] = 0; complete may be NULL); the recorded
 * messages as ONE CSR over (instance, channel): the messages of instance i on channel c
 * are msg_tokens[msg_offsets[r * C + c] .. msg_offsets[r * C + c + 1]), r = i - inst_lo,
 * msg_offsets has (inst_hi - inst_lo) * C + 1 entries.  CL_E_LIMIT (offsets still
 * written) if msg_cap is too small. */
int cl_collect_snapshot_range(cl_sim* sim, int32_t sid, int64_t inst_lo, int64_t inst_hi, int64_t* tokens,
                              int32_t* complete, int64_t* msg_offsets, int64_t* msg_tokens, int64_t msg_cap);
/* CollectSnapshot (sim.go:134-173; finalizeSnapshot node.go:188-195) of instances
 * [inst_lo, inst_hi), packed on the GPU: only the packed arrays cross PCIe.
 *   tokens[(i - inst_lo) * N + rank]    tokenMap (int32), -1 where not complete
 *   complete[i - inst_lo]                1 when the snapshot completed in instance i
 *   msg_offsets[r * C + c]               start of instance r's channel c (int64, (hi-lo)*C+1
 *                                        entries; channels in (src rank, dest rank) order)
 *   msg_tokens[...]                      recorded token counts (int32), delivery order
 * Any output pointer may be NULL; *n_msgs (may be NULL) = messages; CL_E_LIMIT (everything
 * else still written) when msg_cap is too small.  cl_collect_snapshot_range is the same
 * collect with int64 tokens and messages (widened on the host). */
int cl_collect_snapshot_packed(cl_sim* sim, int32_t sid, int64_t inst_lo, int64_t inst_hi, int32_t* tokens,
                               int32_t* complete, int64_t* msg_offsets, int32_t* msg_tokens, int64_t msg_cap,
                               int64_t* n_msgs);
/* Device time of the latest packed collect's kernels (HIP events). */
int cl_collect_time(cl_sim* sim, double* device_ms);
/* Counters over instances (only_ok: restrict to CL_INST_OK instances). */
int cl_get_counters(cl_sim* sim, int32_t only_ok, int64_t* out /* [CL_NUM_COUNTERS] */);
/* Batch checksums computed on the GPU (see CL_SUM_*); all-reduce them across ranks. */
int cl_get_checksums(cl_sim* sim, int64_t* out /* [CL_NUM_SUMS] */);

/* ---- device event trace: the reference's debug Logger (logger.go:12-76) ---- */
/* One LogEvent (logger.go:18-23) per record, in the Logger's order.  Node ranks refer
 * to cl_node_id; `other` is the peer of a Sent/Received record (-1 for Start/End and
 * for a SendTokens to a dest without a link, node.go:121-124); tokens = nodeTokens. */
#define CL_LOG_SENT_TOKEN 0     /* SentMsgRecord, token (node.go:118) */
#define CL_LOG_SENT_MARKER 1    /* SentMsgRecord, marker (node.go:100) */
#define CL_LOG_RECV_TOKEN 2     /* ReceivedMsgRecord, token (sim.go:86) */
#define CL_LOG_RECV_MARKER 3    /* ReceivedMsgRecord, marker (sim.go:86) */
#define CL_LOG_START_SNAPSHOT 4 /* StartSnapshotRecord (sim.go:109) */
#define CL_LOG_END_SNAPSHOT 5   /* EndSnapshotRecord (sim.go:127) */
typedef struct {
  int32_t epoch;  /* Logger.events index = simulator time (sim.go:73, test_common.go:35) */
  int32_t kind;   /* CL_LOG_* */
  int32_t node;   /* LogEvent.nodeId (rank) */
  int32_t other;  /* dest of a Sent record, src of a Received record (rank), else -1 */
  int32_t data;   /* Message.data / snapshot id */
  int32_t tokens; /* LogEvent.nodeTokens */
} cl_log_event;
/* Record the Logger of instances [inst_lo, inst_lo + n_inst) with room for cap events
 * each (n_inst = 0: off, the default).  The next flush replays the program with the
 * trace build of the kernel. */
int cl_trace_enable(cl_sim* sim, int64_t inst_lo, int32_t n_inst, int32_t cap);
/* The Logger of one traced instance: *n_events records, the first min(cap, *n_events)
 * copied to out.  CL_E_LIMIT if the instance emitted more than the enabled capacity. */
int cl_trace_read(cl_sim* sim, int64_t inst, cl_log_event* out, int32_t cap, int32_t* n_events);

/* ---- delay-stream utility (host only) ------------------------------------ */
/* out[i*draws + k] = k-th rand.Intn(5) of rand.Seed(seed_base + i), i in [0, n). */
int cl_go_delay_schedule(int64_t seed_base, int64_t n, int64_t draws, uint8_t* out);
/* Go math/rand Int63 / Intn restatement, for known-answer tests. */
int cl_go_int63(int64_t seed, int64_t n, int64_t* out);
int cl_go_intn(int64_t seed, int32_t bound, int64_t n, int32_t* out);

const char* cl_status_string(int32_t code);
const char* cl_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* CLSNAP_H */
