// cg_engine.h -- data layout shared by the graph engine's host runtime (cg_host.cpp)
// and its gfx950 kernels (cg_kernels.hip).  DESIGN.md §10 draws the same layout.
//
// The graph engine runs ONE reference simulation over a large topology (BASELINE
// configs 4 and 5: 2^20-node regular digraph, 100k-node power-law graph with 4,096
// overlapping snapshots).  State lives in HBM, one entry per node / channel /
// (snapshot, node) / (snapshot, channel); each tick is a short sequence of grid-wide
// phases (pick, marker, expand, tally, scan, push) launched on one HIP stream.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cl_engine.h"  // mix64, status codes

namespace clsnap {

// Counter hash of the synthetic workloads: the same definition is restated in
// oracle/cl_oracle.c (orc_counter_hash) and tests/graphgen.py.
#if defined(__HIPCC__)
__host__ __device__
#endif
inline uint64_t cg_hash(uint64_t seed, uint64_t a, uint64_t b) {
  const uint64_t h = mix64(seed ^ (a * 0x9E3779B97F4A7C15ULL));
  return mix64(h ^ (b * 0xD6E8FEB86659FD93ULL));
}

// FIFO entry (u64): lo32 = payload | kGMarker (token count or snapshot id, common.go:28-31),
// hi32 = receiveTime (sim.go:101).
constexpr uint32_t kGMarker = 0x80000000u;
constexpr uint32_t kGPayload = 0x7fffffffu;
// Recording cursor pair (u64) of (snapshot, in-channel): lo32 = begin, hi32 = end.
constexpr uint32_t kOpen = 0xffffffffu;
// Pending-count accumulator per (snapshot, node): creation adds kBig + links recorded,
// every later marker adds -1; the operation whose result is exactly kBig completes it.
constexpr int32_t kBig = 1 << 30;
constexpr int32_t kGMaxOutDegree = 64;  // non-empty out-channel bitmask per node (u64)
constexpr int32_t kGThreads = 256;      // threads (= nodes) per pick / marker / push block
constexpr int32_t kPushLanes = 4;       // k_push threads per node on small graphs
constexpr int32_t kGStatusHistOverflow = 6;
// A local snapshot created at a node of in-degree above this is expanded over its
// in-links by the whole k_push grid instead of by the creating lane.
constexpr int32_t kSmallIndeg = 64;
// Counters are kept as per-shard partial sums, cpart[shard * kNumCnt + counter]: every
// block adds its block-reduced totals to shard blockIdx % kParts, so no address sees
// more than a few atomics per kernel (a device-scope atomic on one word serializes at
// ~11 ns, MI355X_MICROARCH.md 'fanin').
constexpr int32_t kParts = 512;
enum GCnt : int32_t { GC_PEEK = 0, GC_POP_TOK, GC_POP_MK, GC_PUSH, GC_RECORDED, GC_COMPLETED, kNumCnt = 8 };

// A local snapshot created this tick at a node of in-degree > kSmallIndeg.
struct BigX {
  int32_t lo, hi;  // the node's in-CSR range
  int32_t s0;      // creating sender
  int32_t sid;
  int32_t karr;    // in-position of the arriving channel
  int32_t v;
  int32_t pad[2];
};

// A marker delivered this tick (k_pick -> k_marker).
struct MDel {
  int32_t s0, v, k, sid;  // sender, receiver, in-position of the channel, snapshot id
};

// A delivery that crosses devices in the partitioned mode: sender, receiver, in-position,
// payload word (kGMarker | sid, or token count).
struct PDel {
  int32_t s, v, k;
  uint32_t pay;
};

// Receiver-side channel state is one word per in-channel, tokcnt[k]: the tokens delivered on
// it so far (the recording cursor).  A local snapshot created this tick learns whether its
// in-channel k also delivered this tick, and what, from the SENDER's delivery word: sender
// s = in_src[k] popped on out-link in_oj[k] this tick iff pp[s].x == (t << 6) | in_oj[k],
// with payload pp[s].y (each sender delivers at most once per tick, sim.go:90).

constexpr uint32_t kEmpty = 0xffffffffu;  // head receiveTime word of an empty channel

// Per-(snapshot, node) state, one 16-byte record at sid * n + v: every marker handling
// (k_pick's creation bid, k_marker's creation or close, completion) touches one line instead
// of three arrays' (DESIGN.md §10).
struct alignas(16) SNode {
  unsigned long long W;  // creation key: (tick << 32) | creating sender (initiator: | 0xffffffff); ~0 = none
  int32_t cnt;           // pending accumulator (kBig + links recorded, -1 per later marker)
  int32_t stok;          // recorded node tokens (CreateLocalSnapshot, node.go:77)
};

// Device event trace of the graph engine (the reference's debug Logger, logger.go:12-76).
// One record per LogEvent, appended unordered; the host sorts them into the Logger's order
// by (epoch, order, sub) and restores LogEvent.nodeTokens by replaying the token changes the
// records themselves carry (cg_host.cpp cl_graph_trace_read).  Within an epoch (= simulator
// time, Logger.NewEpoch per Tick, sim.go:73) the Logger holds the tick's deliveries in
// sender rank order (sim.go:76-90), then the traffic sends of that step in node order, then
// the host events in program order.
enum : uint32_t { kTrTick = 0u, kTrSend = 1u, kTrHost = 2u };
constexpr uint32_t kTrSubEnd = 0xffffffffu;  // EndSnapshotRecord after the delivery's records
struct GTraceRec {
  int32_t epoch;
  uint32_t order;  // part (bits 31..30) | key: sender rank (tick), node rank (send), op index (host)
  uint32_t sub;    // 0 the delivery / send / start record, 1 + j the broadcast on out-link j, kTrSubEnd
  int32_t kind;    // TK_* (cl_engine.h) == CL_LOG_* (clsnap.h)
  int32_t node, other, data, pad;
};

enum GOpKind : int32_t { GOP_SEND = 1, GOP_SNAP = 2 };
struct GOp {
  int32_t kind, a, b;  // SEND: a = src rank, b = dest rank; SNAP: a = node rank, b = snapshot id
  int32_t n;           // SEND: tokens
};

// Device scalars of one run.
struct GScal {
  unsigned long long draw;  // next delay draw index (sim.go:101 call count)
  unsigned long long base_trig, base_send;  // this tick's draw bases (scan kernel)
  int32_t status;
  int32_t big_n;    // creations at high in-degree nodes this tick
  int32_t time;     // simulator time of the last tick that ran (sim.go:13)
  int32_t skip;     // the drain is over (or hung): launched drain ticks do nothing
  // device-side drain (test_common.go:123-137), evaluated by k_drain_ctl before each tick
  int32_t dphase;   // 0 waiting for completions, 1 the maxDelay+1 extra ticks, 2 done, 3 hang
  int32_t dleft;    // extra ticks left in phase 1
  int32_t dticks;   // ticks spent waiting
  int32_t dcur;     // first snapshot (< the drain's count) not yet complete
  // drain tick i runs with slot i & 1: its time and whether it runs were decided by the
  // previous tick's k_scan (k_drain_begin for the first), so no control kernel per tick
  int32_t dnow;      // time of the last drain tick decided to run
  int32_t dtime[2];
  int32_t dskip[2];
  // parallel send group (k_sg_check -> k_sg_apply)
  int32_t sg_first;              // position of the group's first failing send (INT32_MAX: none)
  int32_t sg_frozen;             // status at the group's start (k_sg_begin): the run was already frozen
  unsigned long long sg_draw0;   // the group's first draw index
  // partitioned mode: this device's tick totals (k_scan), global bases set by the host
  unsigned long long tot_trig, tot_send;
  // draws of the last tick whose k_push scanned its own bases (small graphs, no k_scan):
  // folded into `draw` by the next kernel that reads it (fold_draw), since every k_push block
  // reads `draw` while the tick runs
  unsigned long long draw_pend;
};
enum : int32_t { kDrainWait = 0, kDrainExtra = 1, kDrainDone = 2, kDrainHang = 3 };
constexpr int32_t kTimeFromDevice = -1;  // tick argument -1 - k: drain slot k (time, skip in GScal)
constexpr int32_t kDrainExtraTicks = 6;  // maxDelay + 1 (test_common.go:135-137)  // tick argument: read the tick's time from GScal.time

struct GParams {
  int32_t n, e;
  int32_t cap_log2;  // FIFO slots per channel = 1 << cap_log2
  int32_t s_cap;     // snapshot ids provisioned
  int32_t hist;      // token payload history slots per channel (0: unit payloads)
  int32_t delay_mode;  // 0 counter hash, 1 schedule
  uint64_t delay_seed;
  const uint8_t* sched;
  int64_t sched_len;
  uint64_t traffic_seed;
  uint32_t traffic_thresh;
  int64_t traffic_steps;
  int32_t n_pblocks;  // node blocks = ceil(n / kGThreads)
  int32_t blk_max_out;  // most out-channels of any node block (k_pick's LDS stage size)
  int32_t push_lanes;  // k_push threads per node: 0 = automatic, else forced (1 or kPushLanes)
  // topology (out-CSR channel order = (src rank, dest rank); in-CSR by (dest, src))
  const int32_t* out_off;   // [n+1]
  const int2* route;        // [e] channel c: (dest rank, in-CSR position)
  const int32_t* in_off;    // [n+1]
  const int32_t* in_src;    // [e] src rank at in-position k
  const uint8_t* in_oj;     // [e] out-link index at the sender of in-position k
  // node state
  int32_t* tokens;     // [n]
  // [n] the sender's delivery word: x = (tick << 6) | out-index popped in that tick, y = the
  // payload word of that pop (kGMarker | sid, or token count) -- one 8-byte entry, so a
  // creation's expansion reads one line per in-link's sender, not two
  int2* pp;
  int32_t* ltrig;      // [n] block-local exclusive prefix of triggered broadcasts (draws)
  int32_t* lsend;      // [n] block-local exclusive prefix of traffic sends
  long long* bsum;     // [2 * n_pblocks] block sums (trig, send) -> exclusive block offsets
  int32_t* crn;        // [n] snapshots created at the node this tick
  uint64_t* cre;       // [e] by in-CSR range of the node: (s0 << 32) | sid
  MDel* mlist;         // [n_pblocks * kGThreads] markers delivered, per pick block
  int32_t* mcnt;       // [n_pblocks]
  BigX* big;           // [n] creations at nodes of in-degree > kSmallIndeg this tick
  unsigned long long* cpart;  // [kParts * kNumCnt]
  // channel state
  // [e] lo32: receiveTime of the head packet (kEmpty if the queue is empty),
  //     hi32: ring head (lo16) | packets queued (hi16)
  uint64_t* hq;
  uint64_t* fifo;      // [e << cap_log2]
  uint32_t* tokcnt;    // [e] by in-position: tokens delivered on the channel so far
  uint32_t* histv;     // [e * hist] by in-position
  // snapshot state
  SNode* sn;           // [s_cap * n] per-(snapshot, node) record: creation key, pending accumulator, node tokens
  uint64_t* rec;       // [s_cap * e] by in-position: recording cursors
  int32_t* done;       // [s_cap] node groups complete (p.done[s_cap..] = gdone)
  int32_t* gdone;      // [s_cap * n_pblocks] nodes complete per group of kGThreads ranks
  int32_t* ctick;      // [s_cap] completion tick (-1)
  GScal* sc;
  const GOp* ops;
  // event trace (nullptr: off)
  GTraceRec* trace;
  uint32_t* trace_cnt;
  int32_t trace_cap;
  // Graph-partitioned mode: this device owns node ranks [part_lo, part_hi)
  // = pick blocks [blk_lo, blk_hi) (part_lo a multiple of kGThreads); whole-graph runs own
  // everything (part 0, [0, n)).  Arrays stay graph-sized; a device touches its own rows.
  int32_t part;
  int32_t part_lo, part_hi, blk_lo, blk_hi;
  int32_t pad1;
  PDel* outbox;          // [n] deliveries by owned senders to other devices' receivers
  uint32_t* out_n;       // [4] 0 outbox rows, 1 remote markers, 2 reports
  MDel* rmlist;          // [n] markers delivered to owned receivers by other devices' senders
  int2* reports;         // [n] (s0, outdeg) broadcasts triggered by other devices' senders
  int32_t* trigv;        // [n] broadcasts triggered by owned senders this tick (draws)
  unsigned long long* rdraw;  // [n] first draw of broadcasts triggered by other devices' senders
  // Device-resident exchange (cl_graph_part_dev_*): every exchange step moves
  // fixed-capacity buckets of 16-B rows between device buffers (one bucket per peer rank:
  // a header row {rows, 0, 0, 0} then bk_cap rows), so a tick needs no host round trip.
  // bk_cap bounds every bucket exactly (from the topology: the senders of one rank with a
  // channel into another's nodes).  Null bk_send: the host-staged exchange.
  int32_t bk_world, bk_rank;
  int32_t bk_span;     // node ranks per rank (owner(v) = v / bk_span)
  int32_t bk_cap;      // rows per bucket after its header
  int4* bk_send;       // [bk_world * (bk_cap + 1)] this rank's outgoing buckets
  const int4* bk_recv; // [bk_world * (bk_cap + 1)] bucket q: what rank q sent here
  uint32_t* bk_cnt;    // [bk_world] rows appended to each outgoing bucket
  long long* tot_send;        // [4] this rank's tick totals: triggers, sends, status
  const long long* tot_recv;  // [bk_world * 4] every rank's totals (all-gathered)
};
// Engine status of a device exchange bucket that overflowed its capacity (cannot happen with
// the topology bound; a guard, never a wrong answer).
constexpr int32_t kGStatusXchgOverflow = 7;

// Launchers (cg_kernels.hip); return hipError_t as int.
int cg_launch_reset(const GParams& p, const int32_t* init_tok, void* stream);
int cg_launch_tick(const GParams& p, int32_t t, void* stream);
// Drain (test_common.go:123-137) on the device: reset the drain state for the snapshots
// [0, n_before), then `ticks` x (k_drain_ctl + one tick whose time comes from GScal):
// k_drain_ctl decides on the device whether the tick runs (waiting, then maxDelay+1 extra
// ticks) or is skipped (drain over / hung), so the host checks only once per batch.
int cg_launch_drain_begin(const GParams& p, int32_t time, int32_t n_before, int64_t max_drain, void* stream);
int cg_launch_drain_ticks(const GParams& p, int32_t n_before, int64_t max_drain, int64_t first, int32_t ticks,
                          void* stream);
int cg_launch_drain_end(const GParams& p, void* stream);  // normal ticks run again
int cg_launch_sends(const GParams& p, int32_t t, void* stream);  // step-0 traffic
int cg_launch_hostops(const GParams& p, int32_t time, int32_t op_begin, int32_t op_count, void* stream);
// A run of host sends from pairwise distinct senders, in parallel: no send of the run
// changes another's sender balance or channel, so every send up to the first failing one
// (program order) executes at once with draw index d + position.
int cg_launch_sendgroup(const GParams& p, int32_t time, int32_t op_begin, int32_t op_count, void* stream);
// Partitioned mode, one tick = pick -> [exchange deliveries] -> receive -> [exchange
// reports] -> tally -> [allgather totals] -> bases -> [exchange replies] -> push.
int cg_launch_part_pick(const GParams& p, int32_t t, void* stream);
int cg_launch_part_receive(const GParams& p, int32_t t, const PDel* in, int32_t n_in, void* stream);
int cg_launch_part_tally(const GParams& p, int32_t step, const int2* rep, int32_t n_rep, void* stream);
int cg_launch_part_bases(const GParams& p, int64_t trig_before, int64_t trig_all, int64_t send_before,
                         int64_t send_all, const int32_t* s0, int32_t n, unsigned long long* draw0, void* stream);
int cg_launch_part_push(const GParams& p, int32_t t, int32_t step, const long long* replies, int32_t n, void* stream);
// The same tick with the device-resident exchange (GParams bk_*): pick -> seal deliveries ->
// [all-to-all] -> receive -> seal reports -> [all-to-all] -> tally -> [all-gather totals] ->
// bases + replies -> [all-to-all] -> push.  No host round trip.
int cg_launch_part_dev_seal(const GParams& p, void* stream);
int cg_launch_part_dev_pick(const GParams& p, int32_t t, void* stream);
int cg_launch_part_dev_receive(const GParams& p, int32_t t, void* stream);
int cg_launch_part_dev_tally(const GParams& p, int32_t step, void* stream);
int cg_launch_part_dev_bases(const GParams& p, void* stream);
int cg_launch_part_dev_push(const GParams& p, int32_t t, int32_t step, void* stream);
// Recorded copies on channels still recording at the end (out[0] += ...).
int cg_launch_finish(const GParams& p, int32_t n_sids, unsigned long long* out, void* stream);
// Batch checks (out zeroed by the caller, 3 + n_sids entries): out[0] final node tokens,
// out[1] in-flight token payloads, out[2] digest over completed snapshots,
// out[3 + sid] = snapshot tokens + recorded token payloads of completed snapshot sid.
int cg_launch_checks(const GParams& p, int32_t n_sids, unsigned long long* out, void* stream);

}  // namespace clsnap
