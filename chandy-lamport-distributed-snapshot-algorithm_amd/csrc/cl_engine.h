// cl_engine.h -- data layout shared by the host runtime (cl_host.cpp) and the gfx950
// kernels (cl_kernels.hip).  DESIGN.md §3 draws the same layout.
#pragma once
#include <stdint.h>

namespace clsnap {

// ---- event program ("op tape") ---------------------------------------------
// Every instance executes the same program; ops are read with scalar loads.
enum OpKind : int32_t {
  OP_SEND = 1,   // a = src rank, b = channel (-1: unknown dest), c = tokens  (node.go:112-131)
  OP_SNAP = 2,   // a = node rank, b = snapshot id                          (sim.go:105-123)
  OP_TICK = 3,   // a = number of ticks                                      (sim.go:71-95)
  OP_DRAIN = 4,  // a = max drain ticks, b = extra ticks (maxDelay+1)        (test_common.go:123-137)
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

// ---- per-channel head word (one u32) ---------------------------------------
//   bits 7..0  : LDS ring head slot
//   bits 15..8 : queued packets (LDS ring + HBM spill), <= 255
//   bits 31..16: token packets delivered on the channel so far (recording cursor)
constexpr uint32_t kCountOne = 1u << 8;
constexpr uint32_t kTokDelivOne = 1u << 16;
constexpr int32_t kMaxQueued = 255;
constexpr int32_t kMaxChannelTokens = 65535;

// ---- limits of the small-graph (instance-per-lane) kernel -----------------
constexpr int32_t kMaxSnapshots = 32;   // STARTED bitmask per node
constexpr int32_t kMaxNodes = 255;      // u8 completion counters
constexpr int32_t kWave = 64;
constexpr int32_t kMaxLdsBytes = 160 * 1024;

// Register image saved per instance between launches (regs[r * stride + inst]).
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

// LDS image of one instance, in 32-bit words.  Word k of the lane's instance lives at
// lds[k * 64 + lane]: every lane owns one bank column, so any per-lane index is
// conflict-free (bank = lane mod 32 for ds_read/write_b32).
struct Layout {
  int32_t cap_log2;   // LDS ring slots per channel = 1 << cap_log2
  int32_t ocap_log2;  // HBM spill ring per channel = 1 << ocap_log2 (-1 = none)
  int32_t sp;         // words of u8 pending counters per node = ceil(S_cap / 4)
  int32_t w_fifo, w_chw, w_tok, w_started, w_pend, w_done, words;
};

inline Layout make_layout(int32_t n_nodes, int32_t n_ch, int32_t cap_log2, int32_t ocap_log2,
                          int32_t s_cap) {
  Layout L;
  L.cap_log2 = cap_log2;
  L.ocap_log2 = ocap_log2;
  L.sp = (s_cap + 3) / 4;
  L.w_fifo = 0;
  L.w_chw = n_ch << cap_log2;
  L.w_tok = L.w_chw + n_ch;
  L.w_started = L.w_tok + n_nodes;
  L.w_pend = L.w_started + n_nodes;
  L.w_done = L.w_pend + n_nodes * L.sp;
  L.words = L.w_done + L.sp;
  return L;
}

// Kernel parameters (passed by value).
struct ExecParams {
  int32_t op_begin, op_end;
  int32_t n_nodes, n_ch;
  Layout lay;
  int32_t n_started_before;  // snapshots started by ops before op_begin
  // delays: draw k of an instance is sched[inst * sched_row + k], k < draws
  // (sched is a kernel argument; sched_row is a multiple of 16 for 16-byte windows)
  int64_t draws, sched_row;
  int64_t n_inst, stride;
  int32_t fresh;
  // state / outputs (instance-fastest, [k][stride])
  uint32_t* state;
  int32_t* regs;
  int32_t* snap_tok;   // [S_cap][N]
  uint32_t* snap_rec;  // [S_cap][C]  lo16 = begin, hi16 = end (channel token cursor)
  int32_t* snap_tick;  // [S_cap]
  uint32_t* ovf;       // [C][1 << ocap_log2] spill ring
  uint32_t* ovh;       // [C] spill ring head
};

struct SumParams {
  int32_t n_nodes, n_ch, s_cap, n_sids;
  int64_t n_inst, stride;
  const int32_t* regs;
  const int32_t* snap_tok;
  const uint32_t* snap_rec;
  const int32_t* snap_tick;
  const uint32_t* state;
  Layout lay;
  const int32_t* hist_off;  // [C+1] token history of each channel (shared by all instances)
  const int32_t* hist_val;
  int64_t total_tokens;
  unsigned long long* out;  // [CL_NUM_SUMS]
};

// Topology image (one int32 array, uniform across lanes, passed as a __restrict__
// kernel argument so the kernel reads it through the scalar cache):
//   [0, N]            out_off  channels of sender v are out_off[v] .. out_off[v+1]-1 (dest order)
//   [N+1, N+1+C)      ch_dst   dest rank of channel c
//   next N+1          in_off
//   next C            in_ch    channels into node w, ordered by src rank
//   next N            init_tok
struct TopoView {
  const int32_t* out_off;
  const int32_t* ch_dst;
  const int32_t* in_off;
  const int32_t* in_ch;
  const int32_t* init_tok;
};

// Launchers (cl_kernels.hip); return hipError_t as int.
int launch_exec(const ExecParams& p, const int32_t* topo, const Op* ops, const uint8_t* sched, void* stream);
int launch_checksums(const SumParams& p, void* stream);

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
