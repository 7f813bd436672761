// cl_engine.h -- data layout shared by the host runtime (cl_host.cpp) and the gfx950
// kernels (cl_kernels.hip).  DESIGN.md §3 draws the same layout.
#pragma once
#include <stdint.h>

namespace clsnap {

// ---- event program ("op tape") ---------------------------------------------
// Every instance executes the same program; ops are read with scalar loads.
enum OpKind : int32_t {
  OP_SEND = 1,   // a = src rank, b = out-index at src (-1: unknown dest), c = tokens  (node.go:112-131)
  OP_SNAP = 2,   // a = node rank, b = snapshot id, c = outdeg(a)                   (sim.go:105-123)
  OP_TICK = 3,   // a = number of ticks                                      (sim.go:71-95)
  OP_DRAIN = 4,  // a = max drain ticks, b = extra ticks (maxDelay+1)        (test_common.go:123-137)
  OP_SENDS = 5,  // a = k: the next k ops are OP_SENDs from pairwise distinct senders, run
                 // as one lane-parallel step (device program only; built by the host from
                 // runs of consecutive sends, e.g. one event-file line per node)
};
struct Op {
  int32_t kind, a, b, c;
};

// ---- per-instance status (mirrors CL_INST_* in include/clsnap.h) ----------
enum : int32_t {
  ST_OK = 0,
  ST_FATAL_INSUFFICIENT = 1,
  ST_FATAL_UNKNOWN_DEST = 2,
  ST_FIFO_OVERFLOW = 3,
  ST_HANG = 4,
  ST_DELAY_EXHAUSTED = 5,
};

// ---- packed FIFO entry (one u32) -------------------------------------------
//   bit 31     : marker flag (Message.isMarker, common.go:29)
//   bits 30..16: receiveTime (sim.go:101), simulator time is capped at kMaxTime
//   bits 15..0 : payload (token count or snapshot id, common.go:30)
constexpr uint32_t kMarkerBit = 0x80000000u;
constexpr int32_t kMaxTime = 32767 - 8;      // receiveTime <= time + 5 must fit 15 bits
constexpr int32_t kMaxPayload = 65535;

// ---- per-link column word (one u32, two 16-bit halves accessed separately) ------
//   lo16 = head word of out-link k (sender side):
//     bits 7..0  : LDS ring head slot
//     bits 15..8 : queued packets (LDS ring + HBM spill), <= 255
//   hi16 = recording cursor of in-link k (receiver side): token packets delivered on the
//          channel so far
// Both halves are read and written with 16-bit LDS accesses (ds_read_u16 / ds_write_b16):
// one column word per link instead of two, with no unpacking.
constexpr uint32_t kCountOne = 1u << 8;
constexpr int32_t kMaxQueued = 255;
constexpr int32_t kMaxChannelTokens = 65535;

// ---- limits of the node-parallel kernel -----------------------------------
constexpr int32_t kMaxSnapshots = 32;   // per-node STARTED bitmask
constexpr int32_t kMaxNodes = 64;       // one instance = one segment of a 64-lane wave
constexpr int32_t kMaxDegree = 127;     // 7-bit out-index in a pick word
constexpr int32_t kWave = 64;
constexpr int32_t kWavesPerBlock = 4;
constexpr int32_t kMaxLdsBytes = 160 * 1024;
// Degree bounds up to this unroll the kernel's per-node loops with the in-link words in
// registers (cl_kernels.hip unrolled()); larger ones keep them in the lane's LDS column.
#ifndef CLSNAP_UNROLL_MAX
#define CLSNAP_UNROLL_MAX 4
#endif
constexpr int32_t kUnrollMaxD = CLSNAP_UNROLL_MAX;

// ---- device event trace (the reference's debug Logger, logger.go:12-76) -------
// One 16-byte record per LogEvent.  Records of an instance are appended unordered and
// sorted on the host by (epoch, order), which restates the Logger's sequence:
//   epoch  = simulator time (Logger.NewEpoch per Tick, sim.go:73; test_common.go:35)
//   order  = tick deliveries first, by delivering sender rank (sim.go:76-90): rank << 8 |
//            sub, sub 0 = ReceivedMsgRecord (sim.go:86), 1 + j = SentMsgRecord of the
//            broadcast on out-link j (node.go:100), 255 = EndSnapshotRecord (sim.go:127);
//            then host events (bit 31) by device op index: op << 8 | sub, sub 0 =
//            SentMsgRecord of SendTokens (node.go:118) or StartSnapshotRecord (sim.go:109),
//            1 + j = the snapshot broadcast's SentMsgRecord on out-link j.
enum TraceKind : uint32_t {
  TK_SENT_TOKEN = 0, TK_SENT_MARKER = 1, TK_RECV_TOKEN = 2, TK_RECV_MARKER = 3,
  TK_START = 4, TK_END = 5,
};
constexpr uint32_t kTraceNoLink = 127;  // SendTokens to a dest with no link (node.go:121-124)
struct TraceRec {
  uint32_t w0;     // epoch (bits 15..0) | kind (18..16) | node rank (24..19) | other rank (31..25)
  uint32_t order;
  int32_t data;    // Message.data: tokens or snapshot id
  int32_t tokens;  // LogEvent.nodeTokens: the logged node's tokens at the event
};

// Pick word published by a sender lane each tick (phase A):
//   bit 31 marker, bit 30 valid, bits 22..16 out-index, bits 15..0 payload.
constexpr uint32_t kPickValid = 0x40000000u;

// Per-instance results written at the end of every launch (regs[inst * R_NUM + r]).
enum : int32_t {
  R_TIME = 0,
  R_DRAW = 1,
  R_STATUS = 2,
  R_NDONE = 3,
  R_PEEK = 4,
  R_POP_TOK = 5,
  R_POP_MK = 6,
  R_PUSH = 7,
  R_INFLIGHT_TOK = 8,
  R_NUM = 9,
};

// Per-lane registers kept in the state image between launches.
enum : int32_t {
  G_TOKENS = 0, G_STARTED, G_TIME, G_DRAW, G_STATUS, G_PEEK, G_POP_TOK, G_POP_MK, G_PUSH, G_NUM
};

// LDS of one wave: a small region shared by the wave's lanes, then a private column per
// lane (word k of lane l at lds[col + k * 64 + l]; a lane only indexes its own column, so
// every data-dependent access is conflict-free).
struct Layout {
  int32_t cap_log2;   // LDS ring slots per out-channel = 1 << cap_log2
  int32_t ocap_log2;  // HBM spill ring per channel = 1 << ocap_log2 (-1 = none)
  int32_t od, id;     // max out-degree / in-degree over nodes
  int32_t s_cap;      // snapshot ids provisioned
  int32_t sp;         // u8 counters per node / per instance: words = s_cap / 4 (s_cap % 4 == 0)
  int32_t ipw;        // instances per wave = 64 / N
  // private column (words): FIFO rings, link words (out-link head | in-link cursor),
  // in-link words (degree bounds above kUnrollMaxD), 16-bit trigger entries, u8 pending
  // counters
  int32_t w_fifo, w_lnk, w_int, w_pend, w_trig, priv;
  // shared region (words, after the 64 private columns)
  int32_t x_pick, x_tslot, x_off, x_done, x_ndone, x_acc;
  int32_t x_delay_begin;  // words of the shared region zeroed at start (everything before x_delay)
  int32_t x_delay;        // wave's delay rows staged in LDS (0 = not staged; rows read from HBM)
  int32_t shared;
  int32_t col;  // first word of the private columns (after the shared region)
  int32_t wave_words;
  int32_t wpb;  // waves per workgroup: kWavesPerBlock, fewer when that many waves' state exceeds LDS
  int32_t rw;   // words per node snapshot record (tokens, then one cursor word per in-link; rec_words)
  // state image per instance (words): per node priv + G_NUM, then s_cap done counters + ndone
  int32_t state_words;
};

// The exec kernel's degree bound for max degree d (cl_kernels.hip launch_exec).
inline int32_t degree_bound(int32_t d) {
  int32_t b = d <= 1 ? 1 : d <= 2 ? 2 : d <= 3 ? 3 : 4;
  while (b < d) b <<= 1;
  return b;
}
// Words per node snapshot record: [tokens, cursor of in-link 0, 1, ...].  Unrolled kernels
// write a record with one vector store, so it is padded to a power of two (16 B for the
// degree-3 8nodes topology); the others store word by word into 1 + id words.
inline int32_t rec_words(int32_t dmax, int32_t id) {
  const int32_t D = degree_bound(dmax);
  if (D > kUnrollMaxD) return 1 + id;
  int32_t r = 1;
  while (r < 1 + D) r <<= 1;
  return r;
}

inline Layout make_layout(int32_t n_nodes, int32_t od, int32_t id, int32_t cap_log2, int32_t ocap_log2,
                          int32_t s_cap, int64_t sched_row = 0, int32_t delay_budget_words = 0) {
  Layout L;
  // unrolled kernels: every lane reserves D out- and in-link words, so the private column
  // offsets are compile-time constants of (D, cap_log2) in the specialized kernels (ColumnC)
  const int32_t dmax = od > id ? od : id;
  const int32_t dbound = degree_bound(dmax);
  const bool unr = dbound <= kUnrollMaxD;
  if (unr) od = id = dbound;
  L.cap_log2 = cap_log2;
  L.ocap_log2 = ocap_log2;
  L.od = od;
  L.id = id;
  L.s_cap = s_cap;
  L.sp = (s_cap + 3) / 4;
  L.ipw = n_nodes > 0 ? kWave / n_nodes : 0;
  L.wpb = kWavesPerBlock;
  L.w_fifo = 0;
  L.w_lnk = od << cap_log2;
  L.w_int = L.w_lnk + (od > id ? od : id);
  // in-link words live in registers when the kernel's degree bound is unrolled
  L.w_trig = L.w_int + (unr ? 0 : id);
  L.w_pend = L.w_trig + (id + 1) / 2;  // 16-bit trigger entries, at most id per tick
  L.priv = L.w_pend + L.sp;
  // shared region first (its fixed-size arrays at compile-time offsets 0, 64, 128, 192),
  // then the 64 private columns from word `col`
  L.x_pick = 0;
  L.x_tslot = kWave;
  L.x_off = 2 * kWave;
  L.x_done = 3 * kWave;                      // u8 completion counters per (instance, snapshot)
  L.x_ndone = L.x_done + L.ipw * L.sp;
  L.x_acc = L.x_ndone + L.ipw;
  L.x_delay_begin = L.x_acc + 5 * L.ipw;
  const int64_t delay_words = (int64_t)L.ipw * sched_row / 4;  // sched_row is a multiple of 16
  if (sched_row > 0 && delay_words <= delay_budget_words) {
    L.x_delay = (L.x_delay_begin + 3) / 4 * 4;  // 16-byte aligned
    L.shared = L.x_delay + (int32_t)delay_words;
  } else {
    L.x_delay = 0;
    L.shared = L.x_delay_begin;
  }
  L.col = (L.shared + 3) / 4 * 4;
  L.wave_words = L.col + L.priv * kWave;
  L.rw = rec_words(dmax, id);
  L.state_words = n_nodes * (L.priv + G_NUM) + s_cap + 1;
  return L;
}

// The private column of an unrolled kernel with degree bound D and 1 << CAP ring slots
// (make_layout with od = id = D): compile-time offsets.
template <int D, int CAP>
struct ColumnC {
  static constexpr int32_t w_fifo = 0, w_lnk = D << CAP, w_int = w_lnk + D, w_trig = w_int,
                           w_pend = w_trig + (D + 1) / 2;
};

// ---- instance-per-lane kernel (cl_lanes.h, cl_jit.cpp) ------------------------------
// Small topologies (N <= 16 nodes, every degree <= 4) can run one instance per lane, with the
// topology compiled into the kernel: a node's state lives in registers of fixed slots, only
// the FIFO rings and the delay row live in the lane's LDS column.  The host describes the
// frozen topology here (the JIT generates the kernel's topology type from it); init_tok is
// read by the kernel at its start.
constexpr int32_t kLanesMaxNodes = 16;
constexpr int32_t kLanesMaxDegree = 4;
// AUTO picks the instance-per-lane kernel from this batch size up, for topologies with a
// degree of 2 or more (measured, gpurun_out/r05p, ms per replay node-parallel / lanes: C3
// 8nodes at 2^16 0.153 / 0.201, 2^17 0.289 / 0.232, 2^18 0.533 / 0.452, 2^19 1.055 / 0.925;
// C2's ring (degree 1, the node-parallel kernel's cheapest shape) at 2^17 0.276 / 0.306)
constexpr int64_t kLanesAutoMinInstances = 1 << 17;
struct LanesTopo {
  int32_t ok;                       // the topology fits the kernel (set by the host)
  uint32_t node[kLanesMaxNodes];    // indeg (3..0) | outdeg (7..4) | out_off (15..8)
  uint32_t inl[kLanesMaxNodes];     // in-link j at bits 8j..8j+7: sender rank (3..0) | its out-index (5..4)
  int32_t init_tok[kLanesMaxNodes]; // tokens at the start (readTopologyFile)
  int32_t max_payload;              // largest token count a send of the program moves
  int32_t max_depth;                // most packets the program can ever push on one channel
};

// Kernel parameters (passed by value).
struct ExecParams {
  int32_t op_begin, op_end;
  int32_t n_nodes, n_ch;
  Layout lay;
  int32_t n_started_before;  // snapshots started by ops before op_begin
  int32_t topo_w;            // words per node block of the topology image (3 + max in-degree)
  // delays: draw k of an instance is sched[inst * sched_row + k], k < draws
  int64_t draws, sched_row;
  int64_t n_inst, stride;
  int32_t fresh;       // start from the initial topology state (else resume from `state`)
  int32_t save_state;  // write the resumable state image at the end
  // state: [state_words][stride]; regs: [stride][R_NUM]
  uint32_t* state;
  int32_t* regs;       // [stride][R_NUM] per-instance results
  // outputs, node index fastest so a wave's stores coalesce:
  int32_t* fin_tok;    // [stride][N]          final node tokens
  // [S_cap][stride][N][rw] one record per (snapshot, node), written when the node creates its
  // local snapshot: word 0 = tokenMap entry, word 1 + k = recording cursors of in-link k
  // (lo16 = begin, hi16 = end, the end written when the channel's marker arrives)
  uint32_t* snap_nod;
  int32_t* snap_tick;  // [stride][S_cap]      completion tick or -1 (one row per instance)
  uint32_t* ovf;       // [C][1 << ocap_log2] spill ring
  uint32_t* ovh;       // [C] spill ring head
  // Replay plan (cl_host.cpp build_plan, from the first full run of the same program and
  // delays): nospill -- no instance ever spilled, every launch may take the spill-free
  // kernel; split_slot > 0 -- the slot map puts the spilling instances last and slots
  // [split_slot, n_inst) run on the spill-capable kernel, concurrently.  spill_flag (probe
  // runs): set to 1 for every instance a push spilled to HBM.
  int32_t nospill;
  uint32_t slot_base;  // first slot of this launch's grid
  int64_t split_slot;
  uint8_t* spill_flag;  // [n_inst] or nullptr
  // slot -> instance for a replay (nullptr: slot i runs instance i).  cl_host orders a
  // replay's instances by their final tick so the segments of a wave finish together
  const int32_t* inst_map;
  // event trace of instances [trace_lo, trace_lo + trace_n) (trace kernel build only)
  TraceRec* trace;          // [trace_n][trace_cap]
  uint32_t* trace_cnt;      // [trace_n] records emitted (may exceed trace_cap: overflow)
  const int32_t* ch_dest;   // [C] dest rank of channel c
  int64_t trace_lo;
  int32_t trace_n, trace_cap;
  // the topology in the form the instance-per-lane kernels are generated from (cl_jit.cpp)
  LanesTopo lt;
};

struct SumParams {
  int32_t n_nodes, n_ch, s_cap, n_sids;
  int64_t n_inst, stride;
  const int32_t* regs;
  const int32_t* fin_tok;
  int32_t rw;
  const uint32_t* snap_nod;  // ExecParams::snap_nod
  const int32_t* ch_slot;    // [C] word of channel c in an instance's records: dest * rw + 1 + in-link
  const int32_t* snap_tick;
  const int32_t* hist_off;  // [C+1] token history of each channel (shared by all instances)
  const int32_t* hist_val;
  int64_t total_tokens;
  unsigned long long* out;  // [CL_NUM_SUMS]
};

// Topology image (uint32, uniform per node, read once per lane at kernel start):
//   node v block at v * topo_w (topo_w = 3 + max in-degree): [indeg, outdeg, out_off, in[0..indeg)]
//     in[k] = src rank (bits 7..0) | sender's out-index of this channel (15..8) | channel id (31..16)
//   then init_tok[N] at N * topo_w
// Launchers (cl_kernels.hip); return hipError_t as int.
// The exec kernel's stream and its timing events (hipEvent_t, or null): the events are
// recorded by the dispatch itself (hipExtLaunchKernel), not as packets of their own --
// two hipEventRecord packets per launch cost 5.7 us of C2's 0.182 ms step.
struct ExecLaunch {
  void* stream;
  void* ev_start;
  void* ev_stop;
  void* stream2;  // split replays: the spill-capable part runs here (fork / join events)
  void* ev_fork;
  void* ev_join;
  // split replays back to back (cl_host.cpp): fork = stream2 first waits for the engine
  // stream (new work there since the last fork), join = the engine stream waits for stream2
  // before the stop event (else the join is deferred to the next call that is not a rerun)
  int32_t fork, join;
  // split replays: the spill-capable dispatch records start and stop events of its own (its
  // half may end after the main stream's stop event when the replays are not joined);
  // *stop2_used is set to 1 when they were recorded, and the launch time is the longer half
  void* ev_stop2;
  int32_t* stop2_used;
  void* ev_start2;
};
int launch_exec(const ExecParams& p, const uint32_t* topo, const Op* ops, const uint8_t* sched, const ExecLaunch& L);
// The instance-per-lane kernel (cl_lanes.h, compiled per topology by cl_jit.cpp): lanes_fit
// says whether a launch can take it; launch_lanes runs it (same outputs, state image and replay
// plan as launch_exec; hipErrorInvalidImage when the kernel could not be compiled, lanes_error
// says why); lanes_jit_stats: run-time compilations so far and their total time.
bool lanes_fit(const ExecParams& p);
int launch_lanes(const ExecParams& p, const uint32_t* topo, const Op* ops, const uint8_t* sched, const ExecLaunch& L);
const char* lanes_error();
void lanes_jit_stats(double* compile_ms, int64_t* compiles);
}  // namespace clsnap
#if !defined(__HIPCC_RTC__)
#include <string>
namespace clsnap {
int lanes_compile_only(const ExecParams& p, double* ms, std::string* log);
}  // namespace clsnap
#endif
namespace clsnap {
int launch_checksums(const SumParams& p, void* stream);

// CollectSnapshot (sim.go:134-173) of snapshot `sid` for instances [lo, lo + n), packed on
// the device (cl_kernels.hip): the node records' token words and the recording cursors are
// expanded over the channels' token histories into one CSR over (instance, channel), channels
// in (src rank, dest rank) order, messages in delivery order (finalizeSnapshot node.go:188-195
// per channel).  Only the packed arrays cross PCIe.
struct PackParams {
  int32_t n_nodes, n_ch, s_cap, rw, sid;
  int64_t lo, n, stride;
  const uint32_t* snap_nod;
  const int32_t* snap_tick;
  const int32_t* ch_slot;
  const int32_t* hist_off;  // [C + 1]
  const int32_t* hist_val;
  int32_t* tokens;          // [n][N] tokenMap by rank, -1 where the snapshot has not completed
  int32_t* complete;        // [n]
  long long* count;         // [n + 1] messages per instance -> exclusive prefix (count[n] = total)
  long long* bsum;          // scan scratch: one per block of kScanItems instances
  long long* offsets;       // [n * C + 1]
  int32_t* msgs;            // [total]
};
constexpr int32_t kScanItems = 2048;  // instances per scan block (256 threads x 8)
// count + scan (total left in p.count[n]), then fill: two calls so the host can size msgs.
int launch_pack_count(const PackParams& p, void* stream);
int launch_pack_fill(const PackParams& p, void* stream);
// Recorded message copies (node.go:179-183) over every instance's completed snapshots:
// out[0] all instances, out[1] status-OK instances.
int launch_recorded(const SumParams& p, void* stream);

// Snapshot content hash (shared definition with oracle/cl_oracle.c orc_snapshot_hash).
#if defined(__HIPCC__)
__host__ __device__
#endif
inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

}  // namespace clsnap
