// cg_engine.h -- data layout shared by the graph engine's host runtime (cg_host.cpp)
// and its gfx950 kernels (cg_kernels.hip).  DESIGN.md §10 draws the same layout.
//
// The graph engine runs ONE reference simulation over a large topology (BASELINE
// configs 4 and 5: 2^20-node regular digraph, 100k-node power-law graph with 4,096
// overlapping snapshots).  State lives in HBM, one entry per node / channel /
// (snapshot, node) / (snapshot, channel); each tick is a short sequence of grid-wide
// phases (pick, marker, expand, tally, scan, push) launched on one HIP stream.
#pragma once
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
constexpr int32_t kTallyBlock = 1024;   // nodes per tally/scan block
constexpr int32_t kGStatusHistOverflow = 6;

enum GOpKind : int32_t { GOP_SEND = 1, GOP_SNAP = 2 };
struct GOp {
  int32_t kind, a, b;  // SEND: a = src rank, b = dest rank; SNAP: a = node rank, b = snapshot id
  int32_t n;           // SEND: tokens
};

// Device scalars of one run.
struct GScal {
  unsigned long long draw;  // next delay draw index (sim.go:101 call count)
  unsigned long long push, peek, pop_tok, pop_mk, recorded, completed;
  unsigned long long base_trig, base_send;  // this tick's draw bases (scan kernel)
  int32_t status;
  int32_t mlist_n;  // senders that delivered a marker this tick
  int32_t xl_n;     // local snapshots created by a marker this tick
  int32_t time;     // simulator time of the last tick that ran (sim.go:13)
};

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
  int32_t n_blocks;  // tally blocks = ceil(n / kTallyBlock)
  // topology (out-CSR channel order = (src rank, dest rank); in-CSR by (dest, src))
  const int32_t* out_off;   // [n+1]
  const int32_t* ch_dst;    // [e]
  const int32_t* ch_inpos;  // [e] in-CSR position of channel c
  const int32_t* in_off;    // [n+1]
  const int32_t* in_src;    // [e] src rank at in-position k
  // node state
  int32_t* tokens;     // [n]
  uint64_t* mask;      // [n] non-empty out-channels (bit = out-index)
  int32_t* pick;       // [n] (tick << 6) | out-index popped in that tick
  int32_t* trig;       // [n] by sender: out-degree of the node its marker created a snapshot at
  int32_t* ltrig;      // [n] block-local exclusive prefix of trig
  int32_t* lsend;      // [n] block-local exclusive prefix of traffic sends
  long long* bsum;     // [2 * n_blocks] block sums (trig, send) -> exclusive block offsets
  int32_t* crn;        // [n] snapshots created at the node this tick
  uint64_t* cre;       // [e] by in-CSR range of the node: (s0 << 32) | sid
  int32_t* mlist;      // [n]
  int32_t* xl;         // [n]
  // channel state
  uint32_t* hc;        // [e] head (lo16) | count (hi16)
  uint64_t* fifo;      // [e << cap_log2]
  uint32_t* tokcnt;    // [e] by in-position: tokens delivered so far
  uint64_t* deliv;     // [e] by in-position: (tick << 32) | payload of that tick's delivery
  uint32_t* histv;     // [e * hist] by in-position
  // snapshot state
  uint64_t* W;         // [s_cap * n] creation key: (tick << 32) | creating sender (initiator: | 0xffffffff)
  int32_t* cnt;        // [s_cap * n] pending accumulator
  int32_t* stok;       // [s_cap * n] recorded node tokens
  uint64_t* rec;       // [s_cap * e] by in-position: recording cursors
  int32_t* done;       // [s_cap] nodes complete
  int32_t* ctick;      // [s_cap] completion tick (-1)
  GScal* sc;
  const GOp* ops;
};

// Launchers (cg_kernels.hip); return hipError_t as int.
int cg_launch_reset(const GParams& p, const int32_t* init_tok, void* stream);
int cg_launch_tick(const GParams& p, int32_t t, int32_t lanes_per_creation, void* stream);
int cg_launch_sends(const GParams& p, int32_t t, void* stream);  // step-0 traffic
int cg_launch_hostops(const GParams& p, int32_t time, int32_t op_begin, int32_t op_count, void* stream);
// Recorded copies on channels still recording at the end (out[0] += ...).
int cg_launch_finish(const GParams& p, int32_t n_sids, unsigned long long* out, void* stream);
// Batch checks (out zeroed by the caller, 3 + n_sids entries): out[0] final node tokens,
// out[1] in-flight token payloads, out[2] digest over completed snapshots,
// out[3 + sid] = snapshot tokens + recorded token payloads of completed snapshot sid.
int cg_launch_checks(const GParams& p, int32_t n_sids, unsigned long long* out, void* stream);

}  // namespace clsnap
