// cg_kernels.hip -- gfx950 kernels of the graph engine: one reference simulation over a
// large topology, state in HBM, one tick = four grid-wide phases on one HIP stream.
//
// Reference semantics restated per phase (paths relative to /root/reference/chandy_lamport):
//   k_pick     Tick (sim.go:71-95): time++, every sender scans its out-links in dest
//              order and pops the first due head (at most one per sender, :90).  Picks
//              from tick-start state equal the reference's sequential picks: a push made
//              during tick t is due at >= t+1 and never changes a non-empty queue's head.
//              The scan reads only the per-channel head receiveTime words (contiguous per
//              sender); the FIFO itself is touched only by the pop.  Tokens are applied at
//              once (HandleToken node.go:174-185 is commutative for the token count;
//              recording is the channel cursor tokcnt); markers are staged for k_marker.
//   k_marker   HandleMarker (node.go:149-171): the first marker of snapshot s at node v
//              is the one from the lowest-ranked sender in the earliest tick (atomicMin on
//              the creation key W); it creates the local snapshot (CreateLocalSnapshot
//              node.go:58-84) and triggers the broadcast; later markers close their
//              channel.  Completion (node.go:165-168, sim.go:126-131) is the pending
//              accumulator reaching exactly kBig.  The creating lane also expands the
//              local snapshot over the node's in-links: recording cursors begin at the
//              channel's delivered-token count AT the creating delivery, i.e. tokens
//              delivered in the same tick by lower-ranked senders are before it and those
//              of higher-ranked senders after it; the recorded node tokens likewise.
//              Each block also tallies, for its 256 node ranks, the broadcasts its
//              senders triggered and the next step's traffic sends.
//   k_scan     SendToNeighbors (node.go:97-109) draws one delay per out-link in the
//              reference's global draw order -- triggering senders in rank order, then
//              the next step's sends in rank order: exclusive scan of the block tallies.
//   k_push     Every node pushes onto its own out-channels: the broadcasts of the local
//              snapshots created at it this tick (in creating-sender order), then its
//              send, so FIFO order is the reference's Queue.Push order (queue.go:18-20).
//              The grid then expands local snapshots created at high in-degree nodes.
//   k_hostops  ProcessEvent for host events (sim.go:58-68, SendTokens node.go:112-131,
//              StartSnapshot sim.go:105-123 / node.go:198-212), in program order.
#include <hip/hip_runtime.h>

#include "cg_engine.h"

namespace clsnap {
namespace {

constexpr int kThreads = kGThreads;

__device__ inline uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

__device__ inline unsigned long long wave_sum(unsigned long long x) {
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

// Add a per-lane count to a device counter, one atomic per wave (result kernels only).
__device__ inline void wave_count(unsigned long long* dst, unsigned long long x) {
  x = wave_sum(x);
  if (lane_id() == 0 && x) atomicAdd(dst, x);
}

// Inclusive prefix sum of a 32-bit value over the wave (every lane active): DPP row shifts
// and row broadcasts, no LDS permutes (a 64-bit __shfl tree costs two per step).
__device__ inline uint32_t wave_incl_scan32(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}
__device__ inline uint32_t wave_total32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan32(v), 63);
}

// Exclusive block scan of N 32-bit values per thread (block totals fit 32 bits): one DPP
// wave scan per value, one LDS exchange.  sh: [N * 16].
template <int N>
__device__ inline void block_exclusive_scan_n32(uint32_t (&v)[N], uint32_t (&tot)[N], uint32_t* sh) {
  const int lane = (int)lane_id(), w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint32_t inc[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    inc[i] = wave_incl_scan32(v[i]);
    if (lane == 63) sh[N * w + i] = inc[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < N; ++i) {
    uint32_t pre = 0, t = 0;
    for (int k = 0; k < nw; ++k) {
      pre += k < w ? sh[N * k + i] : 0u;
      t += sh[N * k + i];
    }
    v[i] = pre + inc[i] - v[i];
    tot[i] = t;
  }
  __syncthreads();
}

// block_exclusive_scan2 for values whose block totals fit 32 bits (one tick's triggers and
// sends): DPP wave scans.  sh: [2 * 16].
template <bool TRAIL = true>  // TRAIL: a barrier after the exchange (sh reused at once)
__device__ inline void block_exclusive_scan2_32(uint32_t& a, uint32_t& b, uint32_t& tot_a, uint32_t& tot_b,
                                                uint32_t* sh) {
  const int lane = (int)lane_id(), w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint32_t ia = wave_incl_scan32(a), ib = wave_incl_scan32(b);
  if (lane == 63) {
    sh[2 * w] = ia;
    sh[2 * w + 1] = ib;
  }
  __syncthreads();
  uint32_t pa = 0, pb = 0;
  tot_a = tot_b = 0;
  for (int k = 0; k < nw; ++k) {
    if (k < w) {
      pa += sh[2 * k];
      pb += sh[2 * k + 1];
    }
    tot_a += sh[2 * k];
    tot_b += sh[2 * k + 1];
  }
  if constexpr (TRAIL) __syncthreads();
  a = pa + ia - a;
  b = pb + ib - b;
}

// Block-reduce NV per-thread counts and add them to this block's counter shard.  Every
// thread of the block must call it (it has a barrier).  A thread's counts are small (one
// tick's peeks, pops, pushes of one node), so the wave sums are 32-bit DPP reductions.
template <int NV>
__device__ inline void block_count(const GParams& p, const int (&idx)[NV], unsigned long long (&x)[NV]) {
  __shared__ unsigned long long sh[NV][kGThreads / 64];
  const int w = threadIdx.x >> 6;
  for (int i = 0; i < NV; ++i) {
    const uint32_t t = wave_total32((uint32_t)x[i]);
    if (lane_id() == 0) sh[i][w] = t;
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    unsigned long long t = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += sh[threadIdx.x][k];
    if (t) atomicAdd(&p.cpart[(blockIdx.x & (kParts - 1)) * kNumCnt + idx[threadIdx.x]], t);
  }
}

// Frozen-run check, uniform over the block (a status set by another block of the same
// kernel must not split a block at a barrier).
__device__ inline bool block_frozen(const GParams& p, int32_t targ = 0) {
  __shared__ int s_frozen;
  if (threadIdx.x == 0) s_frozen = p.sc->status | (targ >= 0 ? p.sc->skip : p.sc->dskip[-1 - targ]);
  __syncthreads();
  return s_frozen != 0;
}

// A tick's time: the argument, or its drain slot's (targ = -1 - slot).
__device__ inline int32_t tick_time(const GParams& p, int32_t targ) {
  return targ >= 0 ? targ : p.sc->dtime[-1 - targ];
}

__device__ inline void set_status(GScal* sc, int32_t code) { atomicCAS(&sc->status, 0, code); }

// The draw counter after a tick whose k_push scanned its own bases (GScal::draw_pend): one
// thread of the next kernel that reads `draw` folds the pending count in first.
__device__ inline void fold_draw(GScal* sc) {
  const unsigned long long d = sc->draw_pend;
  if (d) {
    sc->draw += d;
    sc->draw_pend = 0;
  }
}

// Append one Logger record (trace runs only; one device counter: a debugging aid for
// graphs of modest size).
__device__ inline void gtrace(const GParams& p, int32_t epoch, uint32_t part, uint32_t key, uint32_t sub, int32_t kind,
                              int32_t node, int32_t other, int32_t data) {
  if (!p.trace) return;
  const uint32_t slot = atomicAdd(p.trace_cnt, 1u);
  if (slot < (uint32_t)p.trace_cap)
    p.trace[slot] = GTraceRec{epoch, (part << 30) | (key & 0x3fffffffu), sub, kind, node, other, data, 0};
}

// GetReceiveTime (sim.go:100-102) for draw index k at simulator time `time`.
__device__ inline uint32_t receive_time(const GParams& p, uint64_t k, int32_t time) {
  uint32_t d;
  if (p.delay_mode == 0) {
    d = (uint32_t)((cg_hash(p.delay_seed, k, 0) >> 32) % 5u);
  } else if ((int64_t)k < p.sched_len) {
    d = p.sched[k];
  } else {
    set_status(p.sc, ST_DELAY_EXHAUSTED);
    d = 0;
  }
  return (uint32_t)time + 1u + d;
}

// Queue.Push (queue.go:18-20) onto channel c.
__device__ inline void push_entry(const GParams& p, int32_t c, uint32_t payload, uint32_t rt,
                                  unsigned long long& pushes) {
  const uint64_t q = p.hq[c];
  const uint32_t hc = (uint32_t)(q >> 32);
  const uint32_t head = hc & 0xffffu, cnt = hc >> 16, cap = 1u << p.cap_log2;
  if (cnt >= cap) {
    set_status(p.sc, ST_FIFO_OVERFLOW);
    return;
  }
  p.fifo[((size_t)c << p.cap_log2) + ((head + cnt) & (cap - 1))] = ((uint64_t)rt << 32) | payload;
  p.hq[c] = ((uint64_t)(head | ((cnt + 1) << 16)) << 32) | (cnt == 0 ? rt : (uint32_t)q);
  ++pushes;
}

// The synthetic traffic decision of node v at step `step` (orc_traffic_sends).
__device__ inline bool traffic_send(const GParams& p, int64_t step, int32_t v, int32_t od, int32_t tok,
                                    int32_t* j) {
  if (step >= p.traffic_steps || tok <= 0 || od == 0) return false;
  const uint64_t x = cg_hash(p.traffic_seed, (uint64_t)step, (uint64_t)v);
  if ((uint32_t)x >= p.traffic_thresh) return false;
  *j = (int32_t)(((x >> 32) * (uint64_t)od) >> 32);
  return true;
}

// Append one row to the outgoing exchange bucket of rank q (partitioned mode, device
// exchange).  The capacity is the topology's exact bound; a row past it freezes the run.
__device__ inline void bucket_row(const GParams& p, int32_t q, int4 row) {
  const uint32_t slot = atomicAdd(&p.bk_cnt[q], 1u);
  if (slot < (uint32_t)p.bk_cap) p.bk_send[(size_t)q * (p.bk_cap + 1) + 1 + slot] = row;
  else set_status(p.sc, kGStatusXchgOverflow);
}

// NotifyCompletedSnapshot (sim.go:126-131) for every lane with `done` (node v complete
// in snapshot sid).  Two-level count, so no word sees more than a few hundred atomics: a
// node completes its group of kGThreads node ranks, the group that fills completes one
// of the snapshot's n_pblocks groups, and the add that fills the last one completes the
// snapshot (one word per snapshot hit by every completing wave serialized a whole tick
// behind it: ~16k same-address atomics at ~11 ns when a C4 snapshot sweeps the graph).
__device__ inline void complete_nodes(const GParams& p, bool done, int32_t sid, int32_t v, int32_t t,
                                      unsigned long long& completed) {
  if (!done) return;
  const int32_t g = v / kGThreads;
  const int32_t gsize = min(kGThreads, p.n - g * kGThreads);
  if (atomicAdd(&p.gdone[(size_t)sid * p.n_pblocks + g], 1) + 1 != gsize) return;
  // (partitioned mode: this device's groups; the host joins the devices' completions)
  if (atomicAdd(&p.done[sid], 1) + 1 == p.blk_hi - p.blk_lo) {
    p.ctick[sid] = t;
    ++completed;
  }
}

// ---------------------------------------------------------------------------
// block exclusive scan of (a, b) pairs over blockDim.x threads (multiple of 64)
// ---------------------------------------------------------------------------
template <bool TRAIL>
__device__ inline void block_exclusive_scan2_32(uint32_t& a, uint32_t& b, uint32_t& tot_a, uint32_t& tot_b,
                                                uint32_t* sh);

// Block tally of node rank v = blockIdx.x * kGThreads + threadIdx.x: `trig` draws
// triggered by v's delivery this tick, and v's traffic send of step `step`.
// The node's traffic-send bit for the tally (loads issued by the caller at kernel start,
// ahead of the block's first barrier).
__device__ inline int32_t tally_send_bit(const GParams& p, int32_t b, int32_t step) {
  const int v = b * kGThreads + threadIdx.x;
  int32_t j;
  return v < p.n && traffic_send(p, step, v, p.out_off[v + 1] - p.out_off[v], p.tokens[v], &j) ? 1 : 0;
}

// The tally of a block without broadcast triggers (no marker delivered by its senders):
// the send bits' exclusive prefix from ballots, one barrier.
__device__ inline void tally_sends(const GParams& p, int32_t bk, int32_t sendbit) {
  __shared__ int s_w[kGThreads / 64];
  const int v = bk * kGThreads + threadIdx.x, w = threadIdx.x >> 6;
  const unsigned long long m = __ballot(sendbit != 0);
  const uint32_t lane = lane_id();
  const int excl = __popcll(m & ((1ull << lane) - 1ull));
  if (lane == 0) s_w[w] = __popcll(m);
  __syncthreads();
  int pre = 0, tot = 0;
  for (int k = 0; k < (int)(blockDim.x >> 6); ++k) {
    pre += k < w ? s_w[k] : 0;
    tot += s_w[k];
  }
  if (sendbit) p.lsend[v] = pre + excl;
  if (threadIdx.x == 0) {
    p.bsum[2 * bk] = 0;
    p.bsum[2 * bk + 1] = tot;
  }
}

__device__ inline void tally(const GParams& p, int32_t bk, int32_t trig, int32_t sendbit) {
  // (a block's totals fit 32 bits: its trigger draws are out-degrees, an int32 CSR span, and its
  // sends one per node)
  __shared__ uint32_t sh[2 * (kGThreads / 64)];
  const int v = bk * kGThreads + threadIdx.x;
  uint32_t a = (uint32_t)trig, b = (uint32_t)sendbit, ta, tb;
  block_exclusive_scan2_32(a, b, ta, tb, sh);
  if (trig) p.ltrig[v] = (int32_t)a;
  if (sendbit) p.lsend[v] = (int32_t)b;
  if (threadIdx.x == 0) {
    p.bsum[2 * bk] = ta;
    p.bsum[2 * bk + 1] = tb;
  }
}

// Expand a local snapshot created at v by s0's marker over in-links [lo, hi) (stride
// `step`): cursor pairs, and the token payloads delivered after the creating marker.
__device__ inline int expand_range(const GParams& p, int32_t t, int32_t s0, int32_t sid, int32_t karr,
                                   int32_t lo, int32_t hi, int32_t step) {
  int tsum = 0;
  uint64_t* rec = p.rec + (size_t)sid * p.e;
  for (int32_t k = lo; k < hi; k += step) {
    uint32_t b = p.tokcnt[k];
    bool closed = k == karr;  // the arriving channel does not record (node.go:66-69)
    const int32_t src = p.in_src[k];
    // (pick and payload loaded together: one dependent round trip after in_src, not two)
    const int2 dw = p.pp[src];
    const int32_t pk = dw.x;
    const uint32_t pay = (uint32_t)dw.y;
    if (src > s0 && pk == ((t << 6) | (int32_t)p.in_oj[k])) {  // a later delivery this tick
      if (!(pay & kGMarker)) {
        b -= 1;  // delivered after the creating marker: recorded
        tsum += (int)pay;
      } else if ((int32_t)(pay & kGPayload) == sid) {
        closed = true;  // its own marker arrives later in the same tick
      }
    }
    rec[k] = (uint64_t)b | ((uint64_t)(closed ? b : kOpen) << 32);
  }
  return tsum;
}

// ---------------------------------------------------------------------------
// device-side drain (test_common.go:123-137)
// ---------------------------------------------------------------------------
// The reference's loop `select { case <-getSnapshots: ...; default: sim.Tick() }` until every
// snapshot started before the drain was collected, then maxDelay+1 more ticks: decided for
// the NEXT drain tick into `slot` (one thread).  Completion is checked before the tick, as
// the host loop did -- completions happen in k_marker, before k_scan decides; snapshot
// completions are permanent, so a cursor over [0, n_before) makes the check O(1) amortized.
// A run that needs more than max_drain waiting ticks hangs (status HANG on the host) -- the
// reference would loop forever.
__device__ inline void drain_decide(const GParams& p, int32_t n_before, int32_t max_drain, int32_t slot) {
  GScal* sc = p.sc;
  if (sc->status) {
    sc->dskip[slot] = 1;
    return;
  }
  int32_t ph = sc->dphase;
  if (ph == kDrainWait) {
    int32_t c = sc->dcur;
    while (c < n_before && p.ctick[c] >= 0) ++c;
    sc->dcur = c;
    if (c == n_before) {
      ph = kDrainExtra;
      sc->dleft = kDrainExtraTicks;
    } else if (sc->dticks >= max_drain) {
      sc->dphase = kDrainHang;
      sc->dskip[slot] = 1;
      return;
    } else {
      sc->dticks += 1;
      sc->dtime[slot] = ++sc->dnow;  // time++ of the tick that follows (sim.go:72)
      sc->dskip[slot] = 0;
      return;
    }
  }
  if (ph == kDrainExtra && sc->dleft > 0) {
    sc->dleft -= 1;
    sc->dphase = ph;
    sc->dtime[slot] = ++sc->dnow;
    sc->dskip[slot] = 0;
    return;
  }
  if (ph == kDrainExtra) ph = kDrainDone;
  sc->dphase = ph;
  sc->dskip[slot] = 1;
}

__global__ void k_drain_begin(GParams p, int32_t time, int32_t n_before, int32_t max_drain) {
  GScal* sc = p.sc;
  sc->dphase = kDrainWait;
  sc->dleft = 0;
  sc->dticks = 0;
  sc->dcur = 0;
  sc->skip = 0;
  sc->dnow = time;
  drain_decide(p, n_before, max_drain, 0);  // the first drain tick
}

__global__ void k_drain_end(GParams p) { p.sc->skip = 0; }

// ---------------------------------------------------------------------------
// reset
// ---------------------------------------------------------------------------
__global__ void k_reset(GParams p, const int32_t* init_tok) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < (size_t)p.n) {
    p.tokens[i] = init_tok[i];
    p.pp[i].x = -1;
    p.crn[i] = 0;
  }
  if (i < (size_t)p.e) {
    p.tokcnt[i] = 0u;
    p.hq[i] = kEmpty;
  }
  if (i < (size_t)p.s_cap) p.ctick[i] = -1;
}

// Per-(snapshot, node) records: W = ~0 (no creation), cnt = 0; stok is left as it is (written
// at creation; a poisoned plane stays poisoned where a run writes nothing).  One 12-byte store.
__global__ void __launch_bounds__(kGThreads) k_sn_reset(SNode* sn, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint3* w = reinterpret_cast<uint3*>(&sn[i]);
    *w = make_uint3(0xffffffffu, 0xffffffffu, 0u);
  }
}

// ---------------------------------------------------------------------------
// tick phase A: pick + deliver
// ---------------------------------------------------------------------------
// STAGE head words staged per sender: 8 when every block has at most 8 * kGThreads
// out-channels (16 KB of LDS: ten blocks per CU, C4), else 12 (24 KB; channels past the
// stage are read from HBM by their sender).  C4: 9.35 -> 9.23 ms with 8; C5's hub blocks
// are faster with 12.
template <int STAGE>
__global__ void __launch_bounds__(kGThreads) k_pick(GParams p, int32_t targ) {
  __shared__ int s_m;
  const int32_t t = tick_time(p, targ);  // (drain ticks: decided by the previous tick's k_scan)
  // Head receiveTime words of the block's senders: the block's out-channels are one
  // contiguous CSR range, loaded once with coalesced loads (a lane-per-sender prefetch
  // touched 64 separate 64 B segments per wave instruction).  Channels past kStage
  // (blocks of unusually high out-degree) are read from HBM by their sender.
  constexpr int kStage = kGThreads * STAGE;
  __shared__ uint64_t s_hq[kStage];
  const int bk = p.blk_lo + (int)blockIdx.x;  // (the owned blocks in the partitioned mode)
  const int s = bk * kGThreads + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x == 0) fold_draw(p.sc);  // (the previous tick's draws)
  const int32_t blo = p.out_off[bk * kGThreads];
  const int32_t bhi = p.out_off[min((bk + 1) * kGThreads, p.n)];
  const int32_t nst = min(bhi - blo, kStage);
  int32_t base = 0, od = 0;
  if (s < p.n) {
    base = p.out_off[s];
    od = p.out_off[s + 1] - base;
  }
  // all stage loads issued before the first LDS store (one HBM latency, not one per
  // stride), and before the status check: topology, head words and the check overlap
  constexpr int kPer = kStage / kGThreads;
  uint64_t tmp[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int32_t i = threadIdx.x + k * kGThreads;
    tmp[k] = i < nst ? p.hq[blo + i] : 0;
  }
  // the status check shares the stage's barrier (block_frozen's rule: one value per block)
  __shared__ int s_frozen;
  if (threadIdx.x == 0) {
    s_frozen = p.sc->status | (targ >= 0 ? p.sc->skip : p.sc->dskip[-1 - targ]);
    s_m = 0;
  }
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int32_t i = threadIdx.x + k * kGThreads;
    if (i < nst) s_hq[i] = tmp[k];
  }
  __syncthreads();
  if (s_frozen) return;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    p.sc->time = t;  // time++ (sim.go:72)
    p.sc->big_n = 0;
  }
  unsigned long long c[3] = {0, 0, 0};  // peek, pop_tok, pop_mk
  if (s < p.n) {
    for (int j = 0; j < od; ++j) {
      const int32_t li = base + j - blo;
      const uint64_t q = li < kStage ? s_hq[li] : p.hq[base + j];
      const uint32_t rt = (uint32_t)q;
      if (rt == kEmpty) continue;
      ++c[0];  // Queue.Peek, sim.go:83
      if (rt > (uint32_t)t) continue;
      const int32_t ch = base + j;
      const uint32_t hc = (uint32_t)(q >> 32), capm = (1u << p.cap_log2) - 1;
      const uint32_t head = hc & 0xffffu, cnt = (hc >> 16) - 1;
      const size_t ring = (size_t)ch << p.cap_log2;
      const int2 rte = p.route[ch];
      const uint32_t pay = (uint32_t)p.fifo[ring + head];
      const uint32_t nrt = cnt ? (uint32_t)(p.fifo[ring + ((head + 1) & capm)] >> 32) : kEmpty;
      p.hq[ch] = ((uint64_t)(((head + 1) & capm) | (cnt << 16)) << 32) | nrt;
      p.pp[s] = make_int2((t << 6) | j, (int)pay);
      const int32_t v = rte.x, k = rte.y;
      ++c[(pay & kGMarker) ? 2 : 1];
      if (v < p.part_lo || v >= p.part_hi) {  // partitioned: the receiver's device applies it
        if (p.bk_send) bucket_row(p, v / p.bk_span, make_int4(s, v, k, (int)pay));
        else p.outbox[atomicAdd(&p.out_n[0], 1u)] = PDel{s, v, k, pay};
        break;
      }
      // ReceivedMsgRecord (sim.go:86)
      gtrace(p, t, kTrTick, (uint32_t)s, 0u, (pay & kGMarker) ? TK_RECV_MARKER : TK_RECV_TOKEN, v, s,
             (int32_t)(pay & kGPayload));
      if (pay & kGMarker) {
        const int32_t sid = (int32_t)(pay & kGPayload);
        atomicMin(&p.sn[(size_t)sid * p.n + v].W, ((unsigned long long)t << 32) | (uint32_t)s);
        p.mlist[bk * kGThreads + atomicAdd(&s_m, 1)] = MDel{s, v, k, sid};
      } else {
        atomicAdd(&p.tokens[v], (int32_t)pay);  // HandleToken node.go:175
        if (p.hist) {
          const uint32_t tc = p.tokcnt[k];
          if (tc < (uint32_t)p.hist) p.histv[(size_t)k * p.hist + tc] = pay;
          else set_status(p.sc, kGStatusHistOverflow);
          p.tokcnt[k] = tc + 1;
        } else {
          // (one pop per sender and tick: k has no other writer; a non-returning add ends
          // the lane's chain at the route load instead of waiting for a cursor read:
          // C4 8.61-8.65 -> 8.61-8.62 ms, C5 4,352-4,367 -> 4,335-4,344 ms, gpurun_out/r04e)
          atomicAdd(&p.tokcnt[k], 1u);
        }
      }
      break;
    }
  }
  const int idx[3] = {GC_PEEK, GC_POP_TOK, GC_POP_MK};
  block_count<3>(p, idx, c);
  if (threadIdx.x == 0) p.mcnt[bk] = s_m;
}

// ---------------------------------------------------------------------------
// tick phase B: the markers delivered by pick block b's senders, and block b's tally
// ---------------------------------------------------------------------------
// REMOTE (partitioned mode): the markers other devices' senders delivered to owned
// receivers (k_part_apply's rmlist), 256 per block; their broadcast triggers are reported
// to the senders' devices.  In the partitioned mode the tally runs after that exchange
// (k_tally), so k_marker only records the triggers.
constexpr int32_t kMarkerPrefetchBelow = 1 << 18;
template <bool REMOTE>
__global__ void __launch_bounds__(kGThreads) k_marker(GParams p, int32_t targ) {
  const int32_t t = tick_time(p, targ);
  const int bk = REMOTE ? (int)blockIdx.x : p.blk_lo + (int)blockIdx.x;
  const MDel* list = REMOTE ? p.rmlist + (size_t)bk * kGThreads : p.mlist + (size_t)bk * kGThreads;
  // the tally's inputs (node tokens after this tick's deliveries, out-degree) and the
  // block's marker count are loaded while the status check is in flight
  const int32_t sendbit = p.part ? 0 : tally_send_bit(p, bk, t);
  const int nm = REMOTE ? min(kGThreads, (int)p.out_n[1] - bk * kGThreads) : p.mcnt[bk];
  if (REMOTE && nm <= 0) return;
  // small graphs (C5: most blocks deliver markers every tick) load the block's marker row
  // with the status check, one latency off a per-tick chain; large ones (C4: mostly none,
  // 1.2 GB per run) read it only when it has entries
  const bool pre = !REMOTE && p.n < kMarkerPrefetchBelow;
  MDel mpre{};
  if (pre) mpre = list[threadIdx.x];
  __shared__ int s_nb, s_base;
  __shared__ int s_trig[kGThreads];
  __shared__ int32_t s_ctsum[kGThreads];
  // (cleared before the status check: its barrier orders them before any use)
  s_trig[threadIdx.x] = 0;
  s_ctsum[threadIdx.x] = 0;
  if (threadIdx.x == 0) s_nb = 0;
  if (block_frozen(p, targ)) return;
  // local snapshots created by this block's markers at nodes of in-degree <= kSmallIndeg,
  // expanded over their in-links by the whole block: (creation, in-link) pairs are
  // numbered by an exclusive prefix over the in-degrees
  __shared__ BigX s_cx[kGThreads];
  __shared__ int32_t s_cpre[kGThreads];
  __shared__ uint32_t s_sh[4 * (kGThreads / 64)];
  if (!REMOTE && nm == 0 && !p.part) {  // no markers delivered by this block's senders: the tally only
    tally_sends(p, bk, sendbit);
    return;
  }
  unsigned long long c[1] = {0};  // completed (the recorded copies are summed by k_finish)
  bool done = false;
  int32_t sid = 0, vdone = 0;
  int bslot = -1, cslot = -1;
  BigX bx;
  if ((int)threadIdx.x < nm) {
    const MDel m = pre ? mpre : list[threadIdx.x];
    const int32_t s0 = m.s0, v = m.v, k = m.k;
    sid = m.sid;
    vdone = v;
    const size_t sv = (size_t)sid * p.n + v;
    SNode* rn = &p.sn[sv];
    const uint64_t key = rn->W;
    const int32_t lo = p.in_off[v], hi = p.in_off[v + 1];
    if (key == (((uint64_t)t << 32) | (uint32_t)s0)) {
      // first marker: CreateLocalSnapshot(src) + SendToNeighbors (node.go:153-156)
      const int32_t od = p.out_off[v + 1] - p.out_off[v];
      if (!p.part) s_trig[s0 - bk * kGThreads] = od;
      else if (s0 >= p.part_lo && s0 < p.part_hi) p.trigv[s0] = od;  // (one delivery per sender and tick)
      else if (p.bk_send) bucket_row(p, s0 / p.bk_span, make_int4(s0, od, 0, 0));
      else p.reports[atomicAdd(&p.out_n[2], 1u)] = make_int2(s0, od);
      if (p.trace)  // SendToNeighbors' SentMsgRecords (node.go:100)
        for (int32_t j = p.out_off[v]; j < p.out_off[v + 1]; ++j)
          gtrace(p, t, kTrTick, (uint32_t)s0, 1u + (uint32_t)(j - p.out_off[v]), TK_SENT_MARKER, v, p.route[j].x, sid);
      // (both returning atomics issued before either result is used: one round trip)
      const int add = kBig + (hi - lo) - 1;
      const int slot = atomicAdd(&p.crn[v], 1);
      const int cold = atomicAdd(&rn->cnt, add);
      p.cre[lo + slot] = ((uint64_t)(uint32_t)s0 << 32) | (uint32_t)sid;
      bx = BigX{lo, hi, s0, sid, k, v, {0, 0}};
      if (hi - lo <= kSmallIndeg) {
        cslot = 0;  // numbered below
      } else {
        rn->stok = p.tokens[v];  // k_push's expansion subtracts the later same-tick tokens
        bslot = atomicAdd(&s_nb, 1);
      }
      done = cold + add == kBig;
    } else {
      // later marker: stop recording the channel (node.go:158-160)
      if ((key >> 32) != (uint64_t)t) {  // created in an earlier tick: cursors exist
        const uint32_t e = p.tokcnt[k];
        // (the end cursor only: k_finish sums end - begin when counters are read, so the close
        // does not wait for the begin cursor; C5 3,840-3,870 -> 3,759-3,770 ms per run with the
        // read dropped, gpurun_out/r05am)
        reinterpret_cast<uint32_t*>(&p.rec[(size_t)sid * p.e + k])[1] = e;
      }  // else created this tick by a lower-ranked sender: its expansion closes it
      done = atomicAdd(&rn->cnt, -1) - 1 == kBig;
    }
  }
  if (done && p.trace) {  // EndSnapshotRecord (sim.go:127); the host moves it behind the last marker
    const MDel m = list[threadIdx.x];
    gtrace(p, t, kTrTick, (uint32_t)m.s0, kTrSubEnd, TK_END, vdone, -1, sid);
  }
  complete_nodes(p, done, sid, vdone, t, c[0]);
  const int idx[1] = {GC_COMPLETED};
  block_count<1>(p, idx, c);  // (has a barrier: s_trig and s_nb are final below)
  // one block scan for both: creations numbered in thread order (b), in-link pairs by the
  // prefix of in-degrees (a); and the tally (triggers c, traffic sends d)
  const bool cre = cslot >= 0;
  const int32_t trig = s_trig[threadIdx.x];
  uint32_t sv4[4] = {cre ? (uint32_t)(bx.hi - bx.lo) : 0u, cre ? 1u : 0u, (uint32_t)trig, (uint32_t)sendbit}, tv4[4];
  block_exclusive_scan_n32<4>(sv4, tv4, s_sh);
  const long long a = sv4[0], b = sv4[1], tot = tv4[0], nc = tv4[1];
  if (!p.part) {  // (the partitioned mode tallies after the exchange, k_tally)
    const int v = bk * kGThreads + threadIdx.x;
    if (trig) p.ltrig[v] = (int32_t)sv4[2];
    if (sendbit) p.lsend[v] = (int32_t)sv4[3];
    if (threadIdx.x == 0) {
      p.bsum[2 * bk] = tv4[2];
      p.bsum[2 * bk + 1] = tv4[3];
    }
  }
  if (cre) {
    cslot = (int)b;
    s_cx[cslot] = bx;
    s_cpre[cslot] = (int32_t)a;
  }
  __syncthreads();
  for (int32_t w = threadIdx.x; w < (int32_t)tot; w += kGThreads) {
    int lo = 0, hi = (int)nc - 1;  // last creation j with s_cpre[j] <= w
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_cpre[mid] <= w) lo = mid;
      else hi = mid - 1;
    }
    const BigX& x = s_cx[lo];
    const int32_t kk = x.lo + (w - s_cpre[lo]);
    const int ts = expand_range(p, t, x.s0, x.sid, x.karr, kk, kk + 1, 1);
    if (ts) atomicAdd(&s_ctsum[lo], ts);
  }
  __syncthreads();
  if (cslot >= 0) p.sn[(size_t)bx.sid * p.n + bx.v].stok = p.tokens[bx.v] - s_ctsum[cslot];
  if (threadIdx.x == 0 && s_nb) s_base = atomicAdd(&p.sc->big_n, s_nb);
  __syncthreads();
  if (bslot >= 0) p.big[s_base + bslot] = bx;
}

// The tally alone: the step-0 traffic (before the first tick: no triggers), and in the
// partitioned mode every tick's, with the triggers k_marker and the reports recorded.
__global__ void __launch_bounds__(kGThreads) k_tally(GParams p, int32_t step) {
  const int bk = p.blk_lo + (int)blockIdx.x;
  const int v = bk * kGThreads + threadIdx.x;
  const int32_t sendbit = tally_send_bit(p, bk, step);
  int32_t trig = 0;
  if (p.part && v < p.n) {
    trig = p.trigv[v];
    if (trig) p.trigv[v] = 0;
  }
  if (block_frozen(p)) return;
  tally(p, bk, trig, sendbit);
}

// phase C: exclusive scan of the block tallies (one workgroup, PER entries per thread),
// draw bases
template <int PER>
__global__ void __launch_bounds__(1024) k_scan(GParams p, int32_t targ, int32_t n_before, int32_t max_drain) {
  // the first chunk of block tallies is loaded while the status check is in flight (one
  // latency, not two: this single-workgroup kernel is pure latency, ~6 us per tick)
  long long pa[PER], pb[PER];
  unsigned long long d0 = 0, dp = 0;  // (thread 0: the draw counter, loaded with the tallies)
  if (threadIdx.x == 0 && !p.part) {
    d0 = p.sc->draw;
    dp = p.sc->draw_pend;
  }
  {
    const int i0 = p.blk_lo + PER * threadIdx.x;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const bool in = i0 + q < p.blk_hi;
      pa[q] = in ? p.bsum[2 * (i0 + q)] : 0;
      pb[q] = in ? p.bsum[2 * (i0 + q) + 1] : 0;
    }
  }
  if (block_frozen(p, targ)) {
    if (targ < 0 && threadIdx.x == 0) drain_decide(p, n_before, max_drain, (-1 - targ) ^ 1);  // (stays frozen)
    return;
  }
  __shared__ uint32_t sh[32];
  long long carry_a = 0, carry_b = 0;
  for (int c0 = p.blk_lo; c0 < p.blk_hi; c0 += PER * blockDim.x) {
    const int i0 = c0 + PER * threadIdx.x;
    long long va[PER], vb[PER], a = 0, b = 0;
    for (int q = 0; q < PER; ++q) {
      const bool in = i0 + q < p.blk_hi;
      va[q] = c0 == p.blk_lo ? pa[q] : in ? p.bsum[2 * (i0 + q)] : 0;
      vb[q] = c0 == p.blk_lo ? pb[q] : in ? p.bsum[2 * (i0 + q) + 1] : 0;
      a += va[q];
      b += vb[q];
    }
    uint32_t a32 = (uint32_t)a, b32 = (uint32_t)b, ta, tb;  // (a tick's totals fit 32 bits)
    block_exclusive_scan2_32(a32, b32, ta, tb, sh);
    a = (long long)a32 + carry_a;
    b = (long long)b32 + carry_b;
    for (int q = 0; q < PER; ++q) {
      if (i0 + q < p.blk_hi) {
        p.bsum[2 * (i0 + q)] = a;
        p.bsum[2 * (i0 + q) + 1] = b;
      }
      a += va[q];
      b += vb[q];
    }
    carry_a += ta;
    carry_b += tb;
  }
  if (threadIdx.x == 0 && p.part) {  // the host joins the devices' totals (k_part_bases)
    p.sc->tot_trig = (unsigned long long)carry_a;
    p.sc->tot_send = (unsigned long long)carry_b;
  } else if (threadIdx.x == 0) {
    const unsigned long long d = d0 + dp;  // fold_draw with the prefetched words
    if (dp) p.sc->draw_pend = 0;
    p.sc->base_trig = d;
    p.sc->base_send = d + (unsigned long long)carry_a;
    p.sc->draw = d + (unsigned long long)(carry_a + carry_b);
  }
  if (targ < 0 && threadIdx.x == 0) drain_decide(p, n_before, max_drain, (-1 - targ) ^ 1);  // the next drain tick
}

// The r-th local snapshot created at v this tick in creating-sender order (prev = the
// (r-1)-th): selection over the node's creation slots.
__device__ inline uint64_t next_creation(const GParams& p, int32_t lo, int ncre, int r, uint64_t prev) {
  uint64_t best = ~0ull;
  for (int i = 0; i < ncre; ++i) {
    const uint64_t x = p.cre[lo + i];
    if ((r == 0 || x > prev) && x < best) best = x;
  }
  return best;
}

// A tick's draw bases for k_push: the trigger and send bases and the exclusive block
// prefixes [2 * block] (triggers) / [2 * block + 1] (sends) -- k_scan's (GScal, bsum), or the
// ones a small graph's k_push scans itself into LDS.
struct Bases {
  unsigned long long trig, send;
  const long long* pre;
};
__device__ inline unsigned long long bdraw(const GParams& p, const Bases& b, int32_t s0) {
  if (s0 < p.part_lo || s0 >= p.part_hi) return p.rdraw[s0];  // partitioned: the sender's device replied
  return b.trig + (unsigned long long)b.pre[2 * (s0 / kGThreads)] + (unsigned long long)p.ltrig[s0];
}

// First draw index of the broadcast triggered by sender s0's delivery this tick, and of
// v's traffic send (the scan kernel's block offsets + block-local prefixes).
__device__ inline unsigned long long broadcast_draw(const GParams& p, int32_t s0) {
  if (s0 < p.part_lo || s0 >= p.part_hi) return p.rdraw[s0];  // partitioned: the sender's device replied
  return p.sc->base_trig + (unsigned long long)p.bsum[2 * (s0 / kGThreads)] + (unsigned long long)p.ltrig[s0];
}
__device__ inline unsigned long long send_draw(const GParams& p, int32_t v) {
  return p.sc->base_send + (unsigned long long)p.bsum[2 * (v / kGThreads) + 1] + (unsigned long long)p.lsend[v];
}

// Queue.Push onto a channel whose head word q is held in a register.
__device__ inline void push_q(const GParams& p, int32_t c, uint64_t& q, uint32_t payload, uint32_t rt,
                              unsigned long long& pushes) {
  const uint32_t hc = (uint32_t)(q >> 32);
  const uint32_t head = hc & 0xffffu, cnt = hc >> 16, cap = 1u << p.cap_log2;
  if (cnt >= cap) {
    set_status(p.sc, ST_FIFO_OVERFLOW);
    return;
  }
  p.fifo[((size_t)c << p.cap_log2) + ((head + cnt) & (cap - 1))] = ((uint64_t)rt << 32) | payload;
  q = ((uint64_t)(head | ((cnt + 1) << 16)) << 32) | (cnt == 0 ? rt : (uint32_t)q);
  ++pushes;
}

// k_push for a node with local snapshots created this tick, in chunks of R out-channels:
// a chunk's head words are loaded once as independent loads, every push of the tick onto
// the chunk (broadcasts in creating-sender order, then the traffic send) updates them in
// registers, and they are stored once -- one HBM round trip per chunk instead of a chain
// of one per channel for nodes of high out-degree.  Per channel the push order is the
// reference's (queue.go:18-20); draw indices are the absolute out-link positions.
constexpr int kRegOd = 8;
template <int R>
__device__ inline void push_node_reg(const GParams& p, const Bases& bs, int32_t t, int32_t v, int32_t ob, int32_t od,
                                     int ncre, bool send, int32_t tok, int32_t tj, unsigned long long sd,
                                     int32_t lo, unsigned long long (&c)[2]) {
  p.crn[v] = 0;
  uint32_t srt = 0;
  if (send) {
    // SendTokens(v, out-link tj, 1): node.go:112-131
    p.tokens[v] = tok - 1;
    srt = receive_time(p, sd, t);
  }
  for (int32_t j0 = 0; j0 < od; j0 += R) {
    const int32_t m = od - j0 < R ? od - j0 : R, obc = ob + j0;
    uint64_t q[R];
#pragma unroll
    for (int j = 0; j < R; ++j) q[j] = j < m ? p.hq[obc + j] : 0ull;
    uint64_t prev = 0;
    for (int r = 0; r < ncre; ++r) {
      const uint64_t best = next_creation(p, lo, ncre, r, prev);
      prev = best;
      const int32_t s0 = (int32_t)(best >> 32);
      const uint32_t sid = (uint32_t)best;
      if (r == 0 && s0 < v) {
        // The reference delivers s0's marker before v's own turn in this tick, so v's
        // scan peeks the queues the broadcast makes non-empty (sim.go:82-84).
        const int pk = p.pp[v].x;
        const int pj = (pk >> 6) == t ? (pk & 63) : 64;
#pragma unroll
        for (int j = 0; j < R; ++j)
          if (j < m && j0 + j < pj && (uint32_t)q[j] == kEmpty) ++c[1];
      }
      const unsigned long long draw0 = bdraw(p, bs, s0) + (unsigned long long)j0;
#pragma unroll
      for (int j = 0; j < R; ++j)
        if (j < m) push_q(p, obc + j, q[j], kGMarker | sid, receive_time(p, draw0 + j, t), c[0]);
    }
    if (send) {
#pragma unroll
      for (int j = 0; j < R; ++j)
        if (j0 + j == tj) {
          push_q(p, obc + j, q[j], 1u, srt, c[0]);
          gtrace(p, t, kTrSend, (uint32_t)v, 0u, TK_SENT_TOKEN, v, p.route[obc + j].x, 1);  // node.go:118
        }
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      if (j < m) p.hq[obc + j] = q[j];
    }
  }
}

// k_push with L lanes per node (small graphs: the grid is too small to hide latency with
// one thread per node): lane jl owns out-channels jl, jl + L, ...; each channel gets the
// node's broadcasts in creating-sender order, then the traffic send (queue.go:18-20), so
// per-channel FIFO order is the same as one thread pushing them all.
constexpr int kRegCre = 4;  // creations per node and tick held in registers by push_node_lanes
template <int L>
__device__ inline void push_node_lanes(const GParams& p, const Bases& bs, int32_t t, int32_t v, int32_t ob, int32_t od,
                                       int ncre, bool send, int32_t tok, int32_t tj, unsigned long long sd, int32_t jl,
                                       int32_t lo, unsigned long long (&c)[2]) {
  if (jl == 0) {
    p.crn[v] = 0;
    if (send) p.tokens[v] = tok - 1;  // SendTokens(v, out-link tj, 1): node.go:112-131
  }
  if (ncre <= kRegCre) {
    // the node's creations sorted once into creating-sender order (keys s0 << 32 | sid are
    // distinct: one delivery per sender and tick) with their draw bases loaded together --
    // one cre -> ltrig round trip per node instead of one per channel
    uint64_t cr[kRegCre];
#pragma unroll
    for (int i = 0; i < kRegCre; ++i) cr[i] = i < ncre ? p.cre[lo + i] : ~0ull;
    const int pk = p.pp[v].x;
    auto cswap = [](uint64_t& a, uint64_t& b) {
      const uint64_t x = a < b ? a : b, y = a < b ? b : a;
      a = x;
      b = y;
    };
    cswap(cr[0], cr[1]);
    cswap(cr[2], cr[3]);
    cswap(cr[0], cr[2]);
    cswap(cr[1], cr[3]);
    cswap(cr[1], cr[2]);
    unsigned long long db[kRegCre];
#pragma unroll
    for (int i = 0; i < kRegCre; ++i) db[i] = i < ncre ? bdraw(p, bs, (int32_t)(cr[i] >> 32)) : 0ull;
    // v's own scan peeks the queues the first broadcast made non-empty when its sender
    // delivered before v's turn (sim.go:82-84)
    const bool early = (int32_t)(cr[0] >> 32) < v;
    const int pj = (pk >> 6) == t ? (pk & 63) : 64;
    for (int32_t j = jl; j < od; j += L) {
      uint64_t q = p.hq[ob + j];
      if (early && j < pj && (uint32_t)q == kEmpty) ++c[1];
#pragma unroll
      for (int r = 0; r < kRegCre; ++r)
        if (r < ncre) push_q(p, ob + j, q, kGMarker | (uint32_t)cr[r], receive_time(p, db[r] + (unsigned long long)j, t), c[0]);
      if (send && j == tj) {
        push_q(p, ob + j, q, 1u, receive_time(p, sd, t), c[0]);
        gtrace(p, t, kTrSend, (uint32_t)v, 0u, TK_SENT_TOKEN, v, p.route[ob + j].x, 1);  // node.go:118
      }
      p.hq[ob + j] = q;
    }
    return;
  }
  for (int32_t j = jl; j < od; j += L) {
    uint64_t q = p.hq[ob + j];
    uint64_t prev = 0;
    for (int r = 0; r < ncre; ++r) {
      const uint64_t best = next_creation(p, lo, ncre, r, prev);
      prev = best;
      const int32_t s0 = (int32_t)(best >> 32);
      const uint32_t sid = (uint32_t)best;
      if (r == 0 && s0 < v) {
        // v's own scan peeks the queues s0's broadcast made non-empty (sim.go:82-84)
        const int pk = p.pp[v].x;
        const int pj = (pk >> 6) == t ? (pk & 63) : 64;
        if (j < pj && (uint32_t)q == kEmpty) ++c[1];
      }
      push_q(p, ob + j, q, kGMarker | sid, receive_time(p, bdraw(p, bs, s0) + (unsigned long long)j, t), c[0]);
    }
    if (send && j == tj) {
      push_q(p, ob + j, q, 1u, receive_time(p, sd, t), c[0]);
      gtrace(p, t, kTrSend, (uint32_t)v, 0u, TK_SENT_TOKEN, v, p.route[ob + j].x, 1);  // node.go:118
    }
    p.hq[ob + j] = q;
  }
}

// phase D: every node pushes onto its own out-channels -- the broadcasts of the local
// snapshots created at it this tick (in creating-sender order), then its traffic send;
// then the grid expands the local snapshots created at high in-degree nodes.
// FUSED (graphs of at most kFuseBlocks node blocks, C5): no k_scan launch -- every block
// scans the block tallies itself (2 per thread, L2-resident) into LDS, block 0 leaves the
// tick's draw count in GScal::draw_pend and makes k_scan's drain decision for the next tick
// (completions all happened in k_marker).
constexpr int32_t kFuseBlocks = 2 * kGThreads;
template <int L, bool FUSED>
__global__ void __launch_bounds__(kGThreads) k_push(GParams p, int32_t targ, int32_t sarg, int32_t n_before,
                                                    int32_t max_drain) {
  const int32_t t = tick_time(p, targ);
  const int32_t step = sarg >= 0 ? sarg : t;  // the traffic of step t follows tick t
  const int64_t gid = ((int64_t)p.blk_lo * kGThreads * L) + blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int v = (int)(gid / L), jl = (int)(gid % L);
  int32_t ob = 0, od = 0, ncre = 0, tok = 0, tj = -1, ilo = 0;
  bool send = false;
  uint64_t q0 = 0;
  unsigned long long sd = 0;
  if (v < p.part_hi) {  // loaded while the status check is in flight
    ob = p.out_off[v];
    od = p.out_off[v + 1] - ob;
    ncre = p.crn[v];
    ilo = p.in_off[v];  // (the creation slots' base: off the creation path's load chain)
    tok = p.tokens[v];
    // the traffic decision and what its push reads: the draw index (k_scan's bases, the
    // block tally) and, for a node without broadcasts, the channel's head word
    send = traffic_send(p, step, v, od, tok, &tj);
    if (send) {
      if (!FUSED) sd = send_draw(p, v);
      if (jl == 0) q0 = p.hq[ob + tj];
    }
  }
  // the high in-degree creations to expand at the end (k_marker's count, final before this
  // launch): loaded with the rest, not one round trip after the pushes
  const int nb = p.sc->big_n;
  long long ta0 = 0, tb0 = 0, ta1 = 0, tb1 = 0;  // (FUSED) this thread's two block tallies
  // (FUSED) the draw counter, folded by this tick's k_pick, written by no block of this kernel
  const unsigned long long d0 = FUSED ? p.sc->draw : 0ull;
  if constexpr (FUSED) {
    const int32_t i0 = 2 * (int32_t)threadIdx.x;
    if (i0 < p.n_pblocks) {
      ta0 = p.bsum[2 * i0];
      tb0 = p.bsum[2 * i0 + 1];
    }
    if (i0 + 1 < p.n_pblocks) {
      ta1 = p.bsum[2 * i0 + 2];
      tb1 = p.bsum[2 * i0 + 3];
    }
  }
  if (block_frozen(p, targ)) {
    if (FUSED && targ < 0 && blockIdx.x == 0 && threadIdx.x == 0)
      drain_decide(p, n_before, max_drain, (-1 - targ) ^ 1);  // (stays frozen)
    return;
  }
  Bases bs{0ull, 0ull, p.bsum};
  __shared__ long long s_pre[FUSED ? 2 * kFuseBlocks : 2];
  if constexpr (FUSED) {
    __shared__ uint32_t s_sh[2 * (kGThreads / 64)];
    const int32_t i0 = 2 * (int32_t)threadIdx.x;
    // (the tallies' prefix in one DPP scan; its exchange array is not reused, so the barrier
    // after the s_pre stores is the only one after it)
    uint32_t a32 = (uint32_t)(ta0 + ta1), b32 = (uint32_t)(tb0 + tb1), ta32, tb32;
    block_exclusive_scan2_32<false>(a32, b32, ta32, tb32, s_sh);
    const long long a = a32, b = b32, tot_a = ta32, tot_b = tb32;
    if (i0 < p.n_pblocks) {
      s_pre[2 * i0] = a;
      s_pre[2 * i0 + 1] = b;
    }
    if (i0 + 1 < p.n_pblocks) {
      s_pre[2 * i0 + 2] = a + ta0;
      s_pre[2 * i0 + 3] = b + tb0;
    }
    if (threadIdx.x == 0 && blockIdx.x == 0) {
      p.sc->draw_pend = (unsigned long long)(tot_a + tot_b);
      if (targ < 0) drain_decide(p, n_before, max_drain, (-1 - targ) ^ 1);  // the next drain tick
    }
    __syncthreads();
    bs = Bases{d0, d0 + (unsigned long long)tot_a, s_pre};
    if (send) sd = bs.send + (unsigned long long)s_pre[2 * (v / kGThreads) + 1] + (unsigned long long)p.lsend[v];
  } else {
    bs = Bases{p.sc->base_trig, p.sc->base_send, p.bsum};
  }
  unsigned long long c[2] = {0, 0};  // push, peek
  if (v < p.part_hi) {
    if (ncre) {
      if constexpr (L == 1) push_node_reg<kRegOd>(p, bs, t, v, ob, od, ncre, send, tok, tj, sd, ilo, c);
      else push_node_lanes<L>(p, bs, t, v, ob, od, ncre, send, tok, tj, sd, jl, ilo, c);
    } else if (send && jl == 0) {
      // SendTokens(v, out-link j, 1): node.go:112-131 (one channel: no batching)
      p.tokens[v] = tok - 1;
      push_q(p, ob + tj, q0, 1u, receive_time(p, sd, t), c[0]);
      p.hq[ob + tj] = q0;
      gtrace(p, t, kTrSend, (uint32_t)v, 0u, TK_SENT_TOKEN, v, p.route[ob + tj].x, 1);  // node.go:118
    }
  }
  const int idx[2] = {GC_PUSH, GC_PEEK};
  block_count<2>(p, idx, c);
  // expansion of the local snapshots created at high in-degree nodes: the (creation,
  // in-link) pairs of each staged chunk are numbered by an LDS prefix over in-degrees and
  // dealt round-robin to every thread of the grid
  constexpr int kChunk = 2 * kGThreads;  // descriptors staged in LDS at a time (16 KB)
  __shared__ BigX sx[kChunk];
  __shared__ int32_t spre[kChunk + 1];
  __shared__ uint32_t ssh[2 * (kGThreads / 64)];
  const int64_t gt = blockIdx.x * (int64_t)blockDim.x + threadIdx.x, gs = (int64_t)gridDim.x * blockDim.x;
  for (int c0 = 0; c0 < nb; c0 += kChunk) {
    const int m = nb - c0 < kChunk ? nb - c0 : kChunk;
    __syncthreads();
    const int j0 = 2 * threadIdx.x;
    long long len0 = 0, len1 = 0;
    if (j0 < m) {
      sx[j0] = p.big[c0 + j0];
      len0 = sx[j0].hi - sx[j0].lo;
    }
    if (j0 + 1 < m) {
      sx[j0 + 1] = p.big[c0 + j0 + 1];
      len1 = sx[j0 + 1].hi - sx[j0 + 1].lo;
    }
    // (a chunk's in-degree sum is a span of the int32 in-CSR: 32 bits)
    uint32_t a = (uint32_t)(len0 + len1), z = 0, tot, tz;
    block_exclusive_scan2_32(a, z, tot, tz, ssh);
    spre[j0] = (int32_t)a;
    spre[j0 + 1] = (int32_t)(a + len0);
    if (threadIdx.x == 0) spre[kChunk] = (int32_t)tot;
    __syncthreads();
    for (int64_t w = gt; w < tot; w += gs) {
      int lo = 0, hi = m - 1;  // last j with spre[j] <= w
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (spre[mid] <= w) lo = mid;
        else hi = mid - 1;
      }
      const BigX x = sx[lo];
      const int32_t k = x.lo + (int32_t)(w - spre[lo]);
      const int tsum = expand_range(p, t, x.s0, x.sid, x.karr, k, k + 1, 1);
      if (tsum) atomicSub(&p.sn[(size_t)x.sid * p.n + x.v].stok, tsum);
    }
  }
}

// ---------------------------------------------------------------------------
// host events of one step, in program order (one workgroup)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kGThreads) k_hostops(GParams p, int32_t time, int32_t ob, int32_t oc) {
  __shared__ int s_stop;
  __shared__ unsigned long long s_draw;
  unsigned long long pushes = 0;
  if (threadIdx.x == 0) fold_draw(p.sc);  // (ordered before the loop's first barrier)
  for (int i = 0; i < oc; ++i) {
    const GOp op = p.ops[ob + i];
    // (an L2 read: other threads' pushes may have set the status with an atomic)
    if (threadIdx.x == 0) s_stop = __hip_atomic_load(&p.sc->status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    __syncthreads();
    if (s_stop) break;
    const int32_t v = op.a;
    const int32_t obv = p.out_off[v], od = p.out_off[v + 1] - obv;
    if (op.kind == GOP_SEND) {
      if (threadIdx.x == 0) {
        // SendTokens (node.go:112-131): insufficient tokens, then unknown dest
        if (p.tokens[v] < op.n) {
          set_status(p.sc, ST_FATAL_INSUFFICIENT);
        } else {
          p.tokens[v] -= op.n;
          int32_t lo = 0, hi = od;
          while (lo < hi) {
            const int32_t mid = (lo + hi) >> 1;
            if (p.route[obv + mid].x < op.b) lo = mid + 1;
            else hi = mid;
          }
          const bool link = op.b >= 0 && lo < od && p.route[obv + lo].x == op.b;
          // SentMsgRecord (node.go:118): after the balance check, before the link check
          gtrace(p, time, kTrHost, (uint32_t)(ob + i), 0u, TK_SENT_TOKEN, v, link ? op.b : -1, op.n);
          if (!link) {
            set_status(p.sc, ST_FATAL_UNKNOWN_DEST);
          } else {
            const unsigned long long d = p.sc->draw++;
            push_entry(p, obv + lo, (uint32_t)op.n, receive_time(p, d, time), pushes);
          }
        }
      }
    } else if (v < p.part_lo || v >= p.part_hi) {
      // partitioned: the node's device starts the snapshot; every device counts its draws
      if (threadIdx.x == 0) p.sc->draw += (unsigned long long)od;
    } else {
      // StartSnapshot (sim.go:105-123 -> node.go:198-212): CreateLocalSnapshot("") records
      // every in-link, then SendToNeighbors
      const int32_t sid = op.b;
      const int32_t lo = p.in_off[v], hi = p.in_off[v + 1];
      uint64_t* rec = p.rec + (size_t)sid * p.e;
      for (int32_t k = lo + (int32_t)threadIdx.x; k < hi; k += blockDim.x)
        rec[k] = (uint64_t)p.tokcnt[k] | ((uint64_t)kOpen << 32);
      if (threadIdx.x == 0) {
        gtrace(p, time, kTrHost, (uint32_t)(ob + i), 0u, TK_START, v, -1, sid);  // sim.go:109
        for (int32_t j = 0; j < od && p.trace; ++j)  // SendToNeighbors (node.go:100)
          gtrace(p, time, kTrHost, (uint32_t)(ob + i), 1u + (uint32_t)j, TK_SENT_MARKER, v, p.route[obv + j].x, sid);
        const size_t sv = (size_t)sid * p.n + v;
        p.sn[sv].W = ((uint64_t)(uint32_t)time << 32) | 0xffffffffull;
        p.sn[sv].stok = p.tokens[v];
        atomicAdd(&p.sn[sv].cnt, kBig + (hi - lo));
        s_draw = p.sc->draw;
      }
      __syncthreads();
      // the broadcast's pushes go to distinct channels: one thread per out-link, draw d + j
      const unsigned long long d = s_draw;
      for (int32_t j = threadIdx.x; j < od; j += blockDim.x)
        push_entry(p, obv + j, kGMarker | (uint32_t)sid, receive_time(p, d + j, time), pushes);
      if (threadIdx.x == 0) p.sc->draw = d + od;
    }
    __syncthreads();
  }
  if (pushes) atomicAdd(&p.cpart[GC_PUSH], pushes);
}

// ---------------------------------------------------------------------------
// a run of host sends from pairwise distinct senders (cg_launch_sendgroup)
// ---------------------------------------------------------------------------
// SendTokens' failure of send i (node.go:112-131): 1 insufficient tokens, 2 unknown dest;
// *c = the channel of a send that passes.
__device__ inline int send_check(const GParams& p, const GOp& op, int32_t* c) {
  const int32_t v = op.a;
  if (p.tokens[v] < op.n) return 1;
  const int32_t obv = p.out_off[v], od = p.out_off[v + 1] - obv;
  int32_t lo = 0, hi = od;
  while (lo < hi) {
    const int32_t mid = (lo + hi) >> 1;
    if (p.route[obv + mid].x < op.b) lo = mid + 1;
    else hi = mid;
  }
  if (op.b < 0 || lo >= od || p.route[obv + lo].x != op.b) return 2;
  *c = obv + lo;
  return 0;
}

// Both kernels gate on sg_frozen, the status k_sg_begin saw, never on the live status: the
// group's own first failure sets the status while other blocks of k_sg_apply still have to
// run the sends before it.
__global__ void __launch_bounds__(kGThreads) k_sg_check(GParams p, int32_t ob, int32_t oc) {
  const int32_t i = blockIdx.x * kGThreads + threadIdx.x;
  if (i == 0) p.sc->sg_draw0 = p.sc->draw;
  if (i >= oc || p.sc->sg_frozen) return;
  int32_t c;
  if (send_check(p, p.ops[ob + i], &c)) atomicMin(&p.sc->sg_first, i);
}

__global__ void __launch_bounds__(kGThreads) k_sg_apply(GParams p, int32_t time, int32_t ob, int32_t oc) {
  const int32_t i = blockIdx.x * kGThreads + threadIdx.x;
  unsigned long long pushes = 0;
  if (p.sc->sg_frozen == 0 && i < oc) {
    const int32_t first = p.sc->sg_first;
    const unsigned long long d0 = p.sc->sg_draw0;
    if (i == 0) p.sc->draw = d0 + (unsigned long long)(first < oc ? first : oc);  // draws of the sends that ran
    const GOp op = p.ops[ob + i];
    int32_t c = -1;
    const int fail = i <= first ? send_check(p, op, &c) : 0;
    if (i < first) {  // SentMsgRecord (node.go:118), tokens -= n, Queue.Push with draw d0 + i
      gtrace(p, time, kTrHost, (uint32_t)(ob + i), 0u, TK_SENT_TOKEN, op.a, op.b, op.n);
      p.tokens[op.a] -= op.n;
      push_entry(p, c, (uint32_t)op.n, receive_time(p, d0 + (unsigned long long)i, time), pushes);
    } else if (i == first) {  // the first failure freezes the run exactly where the program does
      if (fail == 1) {
        set_status(p.sc, ST_FATAL_INSUFFICIENT);
      } else {  // logged and debited before the link check (node.go:118-124)
        gtrace(p, time, kTrHost, (uint32_t)(ob + i), 0u, TK_SENT_TOKEN, op.a, -1, op.n);
        p.tokens[op.a] -= op.n;
        set_status(p.sc, ST_FATAL_UNKNOWN_DEST);
      }
    }
  }
  wave_count(&p.cpart[GC_PUSH], pushes);
}

// ---------------------------------------------------------------------------
// graph-partitioned mode: the device halves of the exchange steps
// ---------------------------------------------------------------------------
// Deliveries by other devices' senders to owned receivers: k_pick's receiver half
// (HandleToken node.go:174-185 on the token count and channel cursor; markers keyed and
// staged for k_marker<true>).  Every channel carries at most one delivery per tick.
__device__ inline void apply_delivery(const GParams& p, int32_t t, const PDel d) {
  // the remote sender's delivery word, on this device, for the expansions here
  p.pp[d.s] = make_int2((t << 6) | (int32_t)p.in_oj[d.k], (int)d.pay);
  if (d.pay & kGMarker) {
    const int32_t sid = (int32_t)(d.pay & kGPayload);
    atomicMin(&p.sn[(size_t)sid * p.n + d.v].W, ((unsigned long long)t << 32) | (uint32_t)d.s);
    p.rmlist[atomicAdd(&p.out_n[1], 1u)] = MDel{d.s, d.v, d.k, sid};
  } else {
    atomicAdd(&p.tokens[d.v], (int32_t)d.pay);
    const uint32_t tc = p.tokcnt[d.k];
    if (p.hist) {
      if (tc < (uint32_t)p.hist) p.histv[(size_t)d.k * p.hist + tc] = d.pay;
      else set_status(p.sc, kGStatusHistOverflow);
    }
    p.tokcnt[d.k] = tc + 1;
  }
}

__global__ void __launch_bounds__(kGThreads) k_part_apply(GParams p, int32_t t, const PDel* in, int32_t n_in) {
  const int32_t i = blockIdx.x * kGThreads + threadIdx.x;
  if (i >= n_in || p.sc->status) return;
  apply_delivery(p, t, in[i]);
}

// ---- device exchange (cl_graph_part_dev_*): fixed-capacity buckets, no host round trip ----
// Row r of received bucket q (rows past the bucket's header count do not exist).
__device__ inline bool bucket_in(const GParams& p, int64_t i, int32_t* q, int32_t* r, int4* row) {
  if (i >= (int64_t)p.bk_world * p.bk_cap) return false;
  *q = (int32_t)(i / p.bk_cap);
  *r = (int32_t)(i % p.bk_cap);
  const int4* b = p.bk_recv + (size_t)*q * (p.bk_cap + 1);
  if (*r >= b[0].x) return false;
  *row = b[1 + *r];
  return true;
}

// Seal the outgoing buckets: header row = rows appended (counters reset for the next step).
__global__ void k_bk_seal(GParams p) {
  for (int32_t q = threadIdx.x; q < p.bk_world; q += blockDim.x) {
    const uint32_t c = p.bk_cnt[q];
    p.bk_send[(size_t)q * (p.bk_cap + 1)] = make_int4((int)min(c, (uint32_t)p.bk_cap), 0, 0, 0);
    p.bk_cnt[q] = 0;
  }
}

// Deliveries other devices' senders addressed to owned receivers (k_part_apply's rows).
__global__ void __launch_bounds__(kGThreads) k_bk_apply(GParams p, int32_t t) {
  int32_t q, r;
  int4 d;
  if (p.sc->status || !bucket_in(p, blockIdx.x * (int64_t)kGThreads + threadIdx.x, &q, &r, &d)) return;
  apply_delivery(p, t, PDel{d.x, d.y, d.z, (uint32_t)d.w});
}

// Reports (s0, outdeg) about owned senders whose markers created snapshots on other devices.
__global__ void __launch_bounds__(kGThreads) k_bk_trig(GParams p) {
  int32_t q, r;
  int4 d;
  if (bucket_in(p, blockIdx.x * (int64_t)kGThreads + threadIdx.x, &q, &r, &d)) p.trigv[d.x] = d.y;
}

// This rank's tick totals for the all-gather (k_scan wrote them; a frozen run's are stale,
// its status stops every rank).
__global__ void k_bk_totals(GParams p) {
  p.tot_send[0] = (long long)p.sc->tot_trig;
  p.tot_send[1] = (long long)p.sc->tot_send;
  p.tot_send[2] = p.sc->status;
  p.tot_send[3] = 0;
}

// Global draw bases from every rank's totals (k_part_bases with the sums taken on the
// device); a rank that froze stops every rank at the same step with its status.
__global__ void k_bk_bases(GParams p) {
  long long tb = 0, ta = 0, sb = 0, sa = 0, st = 0;
  for (int32_t r = 0; r < p.bk_world; ++r) {
    const long long* x = p.tot_recv + 4 * r;
    ta += x[0];
    sa += x[1];
    if (r < p.bk_rank) {
      tb += x[0];
      sb += x[1];
    }
    st = max(st, x[2]);
  }
  if (st) {
    if (!p.sc->status) p.sc->status = (int32_t)st;
    return;
  }
  fold_draw(p.sc);
  const unsigned long long d = p.sc->draw;
  p.sc->base_trig = d + (unsigned long long)tb;
  p.sc->base_send = d + (unsigned long long)(ta + sb);
  p.sc->draw = d + (unsigned long long)(ta + sa);
}

// Replies: the first draw of each reported broadcast, back into the reporting rank's bucket
// in report order.  Thread r = 0 of every bucket writes its header.
__global__ void __launch_bounds__(kGThreads) k_bk_draws(GParams p) {
  const int64_t i = blockIdx.x * (int64_t)kGThreads + threadIdx.x;
  if (i >= (int64_t)p.bk_world * p.bk_cap) return;
  const int32_t q = (int32_t)(i / p.bk_cap), r = (int32_t)(i % p.bk_cap);
  const int4* b = p.bk_recv + (size_t)q * (p.bk_cap + 1);
  const int32_t n = b[0].x;
  int4* o = p.bk_send + (size_t)q * (p.bk_cap + 1);
  if (r == 0) o[0] = make_int4(n, 0, 0, 0);
  if (r >= n) return;
  const int32_t s0 = b[1 + r].x;
  const unsigned long long d = broadcast_draw(p, s0);
  o[1 + r] = make_int4(s0, (int)(uint32_t)d, (int)(uint32_t)(d >> 32), 0);
}

// The replies to this rank's reports: first draws of broadcasts on remote senders' markers.
__global__ void __launch_bounds__(kGThreads) k_bk_rdraw(GParams p) {
  int32_t q, r;
  int4 d;
  if (bucket_in(p, blockIdx.x * (int64_t)kGThreads + threadIdx.x, &q, &r, &d))
    p.rdraw[d.x] = (unsigned long long)(uint32_t)d.y | ((unsigned long long)(uint32_t)d.z << 32);
}

// Reports of broadcasts that other devices' receivers created on owned senders' markers.
__global__ void __launch_bounds__(kGThreads) k_part_trig(GParams p, const int2* rep, int32_t n) {
  const int32_t i = blockIdx.x * kGThreads + threadIdx.x;
  if (i < n) p.trigv[rep[i].x] = rep[i].y;
}

// Global draw bases: the triggers of lower devices' senders draw first, then this
// device's; the next step's sends likewise after every trigger (sim.go:101 call order).
__global__ void k_part_bases(GParams p, long long trig_before, long long trig_all, long long send_before,
                             long long send_all) {
  fold_draw(p.sc);
  const unsigned long long d = p.sc->draw;
  p.sc->base_trig = d + (unsigned long long)trig_before;
  p.sc->base_send = d + (unsigned long long)(trig_all + send_before);
  p.sc->draw = d + (unsigned long long)(trig_all + send_all);
}

// First draw of the broadcast each reported sender triggered (the replies).
__global__ void __launch_bounds__(kGThreads) k_part_draws(GParams p, const int32_t* s0, int32_t n,
                                                          unsigned long long* out) {
  const int32_t i = blockIdx.x * kGThreads + threadIdx.x;
  if (i < n) out[i] = broadcast_draw(p, s0[i]);
}

__global__ void __launch_bounds__(kGThreads) k_part_rdraw(GParams p, const long long* rows, int32_t n) {
  const int32_t i = blockIdx.x * kGThreads + threadIdx.x;
  if (i < n) p.rdraw[rows[2 * i]] = (unsigned long long)rows[2 * i + 1];
}

// ---------------------------------------------------------------------------
// results
// ---------------------------------------------------------------------------
// Recorded copies (HandleToken appended them, node.go:179-183) of every created local snapshot:
// end - begin of each closed channel, and the delivered count - begin of a channel still
// recording.
__global__ void k_finish(GParams p, int32_t n_sids, unsigned long long* out) {
  const size_t span = (size_t)(p.part_hi - p.part_lo);  // owned nodes
  const size_t total = (size_t)n_sids * span;
  unsigned long long rec = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int32_t sid = (int32_t)(i / span), v = p.part_lo + (int32_t)(i % span);
    const size_t sv = (size_t)sid * p.n + v;
    if (p.sn[sv].W == ~0ull) continue;
    const uint64_t* r = p.rec + (size_t)sid * p.e;
    for (int32_t k = p.in_off[v]; k < p.in_off[v + 1]; ++k) {
      const uint64_t x = r[k];
      const uint32_t b = (uint32_t)x, e = (uint32_t)(x >> 32);
      rec += (e == kOpen ? p.tokcnt[k] : e) - b;
    }
  }
  wave_count(out, rec);
}

__device__ inline long long hist_sum(const GParams& p, int32_t k, uint32_t b, uint32_t e) {
  if (!p.hist) return (long long)(e - b);
  long long s = 0;
  for (uint32_t q = b; q < e; ++q) s += p.histv[(size_t)k * p.hist + q];
  return s;
}

// State terms: final node tokens (checkTokens, test_common.go:298-302) and tokens still
// in flight.
__global__ void k_checks_state(GParams p, unsigned long long* out) {
  const size_t gt = blockIdx.x * (size_t)blockDim.x + threadIdx.x, gs = (size_t)gridDim.x * blockDim.x;
  unsigned long long fin = 0, infl = 0;
  // (partitioned mode: owned nodes and their out-channels)
  for (size_t v = p.part_lo + gt; v < (size_t)p.part_hi; v += gs) fin += (unsigned long long)(long long)p.tokens[v];
  const uint32_t capm = (1u << p.cap_log2) - 1;
  for (size_t c = p.out_off[p.part_lo] + gt; c < (size_t)p.out_off[p.part_hi]; c += gs) {
    const uint32_t hc = (uint32_t)(p.hq[c] >> 32);
    for (uint32_t q = 0; q < (hc >> 16); ++q) {
      const uint64_t x = p.fifo[(c << p.cap_log2) + (((hc & 0xffffu) + q) & capm)];
      if (!((uint32_t)x & kGMarker)) infl += (uint32_t)x;
    }
  }
  wave_count(&out[0], fin);
  wave_count(&out[1], infl);
}

// Snapshot terms, grid (chunks, sid): cut sum (tokens recorded at nodes + recorded
// message payloads) and the content digest of every completed snapshot.
__global__ void k_checks_snap(GParams p, int32_t n_sids, unsigned long long* out) {
  const size_t gt = blockIdx.x * (size_t)blockDim.x + threadIdx.x, gs = (size_t)gridDim.x * blockDim.x;
  for (int32_t sid = blockIdx.y; sid < n_sids; sid += gridDim.y) {
    if (p.ctick[sid] < 0) continue;
    unsigned long long cut = 0, dig = 0;
    const SNode* sn = p.sn + (size_t)sid * p.n;
    for (size_t v = p.part_lo + gt; v < (size_t)p.part_hi; v += gs) {
      const int32_t st = sn[v].stok;
      dig += mix64(cg_hash(0x5107ull, (uint64_t)sid, (uint64_t)v) ^ (uint64_t)(uint32_t)st);
      cut += (unsigned long long)(long long)st;
    }
    const uint64_t* rec = p.rec + (size_t)sid * p.e;
    for (size_t c = gt; c < (size_t)p.e; c += gs) {
      const int2 rt = p.route[c];
      if (rt.x < p.part_lo || rt.x >= p.part_hi) continue;  // (partitioned: channels into owned nodes)
      const int32_t k = rt.y;
      const uint64_t x = rec[k];
      const uint32_t b = (uint32_t)x, e = (uint32_t)(x >> 32);
      const long long s = hist_sum(p, k, b, e);
      dig += mix64(cg_hash(0xC4A1ull, (uint64_t)sid, (uint64_t)c) ^ (((uint64_t)(e - b) << 32) | (uint32_t)s));
      cut += (unsigned long long)s;
    }
    wave_count(&out[2], dig);
    wave_count(&out[3 + sid], cut);
  }
}

inline int grid_for(int64_t n, int threads = kThreads) { return (int)((n + threads - 1) / threads); }

}  // namespace

int cg_launch_reset(const GParams& p, const int32_t* init_tok, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  {  // per-(snapshot, node) records: no creation, accumulator 0 (stok is written at creation)
    const int64_t nsn = (int64_t)p.s_cap * p.n;
    const int64_t grid = nsn / kThreads + 1 < 65536 ? nsn / kThreads + 1 : 65536;
    hipLaunchKernelGGL(k_sn_reset, dim3((unsigned)grid), dim3(kThreads), 0, s, p.sn, nsn);
    if ((e = hipGetLastError())) return e;
  }
  if ((e = hipMemsetAsync(p.done, 0, (size_t)p.s_cap * (1 + p.n_pblocks) * sizeof(int32_t), s))) return e;
  if ((e = hipMemsetAsync(p.sc, 0, sizeof(GScal), s))) return e;
  if ((e = hipMemsetAsync(p.cpart, 0, (size_t)kParts * kNumCnt * sizeof(unsigned long long), s))) return e;
  int64_t m = p.n > p.e ? p.n : p.e;
  if (p.s_cap > m) m = p.s_cap;
  hipLaunchKernelGGL(k_reset, dim3(grid_for(m)), dim3(kThreads), 0, s, p, init_tok);
  return hipGetLastError();
}

void launch_pick(const GParams& p, dim3 grid, int32_t t, hipStream_t s) {
  if (p.blk_max_out <= 8 * kGThreads) hipLaunchKernelGGL(k_pick<8>, grid, dim3(kGThreads), 0, s, p, t);
  else hipLaunchKernelGGL(k_pick<12>, grid, dim3(kGThreads), 0, s, p, t);
}

// k_push lanes per node: graphs under kLanesBelow nodes (fewer than ~1 wave per SIMD at one
// thread per node) push with kPushLanes threads per node; p.push_lanes forces either path
// (cl_graph_set_push_lanes: the exact-match tests run both on the same graphs).
constexpr int32_t kLanesBelow = 1 << 18;
// (over the owned node blocks [blk_lo, blk_hi): all of them outside the partitioned mode)
// fused: k_push scans the tick's draw bases itself (no k_scan launch; fuse_scan(p)).
template <bool F>
static void launch_push_t(const GParams& p, int32_t t, int32_t step, hipStream_t s, int32_t n_before, int32_t md) {
  const int32_t nb = p.blk_hi - p.blk_lo;
  if (nb <= 0) return;
  if (p.push_lanes ? p.push_lanes == kPushLanes : p.n < kLanesBelow) {
    const int64_t m = (int64_t)(p.part_hi - p.part_lo) * kPushLanes;
    hipLaunchKernelGGL((k_push<kPushLanes, F>), dim3((unsigned)((m + kGThreads - 1) / kGThreads)), dim3(kGThreads), 0, s,
                       p, t, step, n_before, md);
  } else {
    hipLaunchKernelGGL((k_push<1, F>), dim3(nb), dim3(kGThreads), 0, s, p, t, step, n_before, md);
  }
}
void launch_push(const GParams& p, int32_t t, int32_t step, hipStream_t s) { launch_push_t<false>(p, t, step, s, 0, 0); }
void launch_push(const GParams& p, int32_t t, hipStream_t s) { launch_push(p, t, t, s); }
// Small whole-graph runs fold the scan into k_push (C5: 391 node blocks; one launch and its
// boundary less per tick); large ones keep k_scan (C4: 4,096 tallies per block would be
// 64 KB of L2 reads per k_push block).
static bool fuse_scan(const GParams& p) { return !p.part && p.n_pblocks <= kFuseBlocks; }

// k_scan on a per-tick latency path: up to 512 block tallies (C5: 391) are scanned by one
// wave, eight per thread; more by whole waves of four per thread, at most 1024 threads
// (C5 with a 1024-thread workgroup: 5,242 ms per run; 2 waves: 5,038)
static void launch_scan(const GParams& p, int32_t targ, int32_t n_before, int32_t max_drain, hipStream_t s) {
  const int32_t nb = p.blk_hi - p.blk_lo;
  if (nb <= 8 * 64) {
    hipLaunchKernelGGL(k_scan<8>, dim3(1), dim3(64), 0, s, p, targ, n_before, max_drain);
    return;
  }
  const int32_t th = ((nb + 3) / 4 + 63) & ~63;
  hipLaunchKernelGGL(k_scan<4>, dim3(1), dim3((unsigned)(th > 1024 ? 1024 : th)), 0, s, p, targ, n_before, max_drain);
}

int cg_launch_sends(const GParams& p, int32_t t, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_tally, dim3(p.n_pblocks), dim3(kGThreads), 0, s, p, t);
  launch_scan(p, 0, 0, 0, s);
  launch_push(p, t, s);
  return hipGetLastError();
}

int cg_launch_tick(const GParams& p, int32_t t, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  launch_pick(p, dim3(p.n_pblocks), t, s);
  hipLaunchKernelGGL(k_marker<false>, dim3(p.n_pblocks), dim3(kGThreads), 0, s, p, t);
  if (fuse_scan(p)) {
    launch_push_t<true>(p, t, t, s, 0, 0);
  } else {
    launch_scan(p, t, 0, 0, s);
    launch_push(p, t, s);
  }
  return hipGetLastError();
}

int cg_launch_drain_begin(const GParams& p, int32_t time, int32_t n_before, int64_t max_drain, void* stream) {
  const int32_t md = max_drain > INT32_MAX ? INT32_MAX : (int32_t)max_drain;
  hipLaunchKernelGGL(k_drain_begin, dim3(1), dim3(1), 0, (hipStream_t)stream, p, time, n_before, md);
  return hipGetLastError();
}

// Drain ticks first .. first + ticks - 1 of this drain: tick i reads its time and whether it
// runs from slot i & 1, and its k_scan decides tick i + 1 into the other slot.
int cg_launch_drain_ticks(const GParams& p, int32_t n_before, int64_t max_drain, int64_t first, int32_t ticks,
                          void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int32_t md = max_drain > INT32_MAX ? INT32_MAX : (int32_t)max_drain;
  for (int32_t i = 0; i < ticks; ++i) {
    const int32_t ta = -1 - (int32_t)((first + i) & 1);
    launch_pick(p, dim3(p.n_pblocks), ta, s);
    hipLaunchKernelGGL(k_marker<false>, dim3(p.n_pblocks), dim3(kGThreads), 0, s, p, ta);
    if (fuse_scan(p)) {
      launch_push_t<true>(p, ta, ta, s, n_before, md);
    } else {
      launch_scan(p, ta, n_before, md, s);
      launch_push(p, ta, ta, s);
    }
  }
  return hipGetLastError();
}

int cg_launch_drain_end(const GParams& p, void* stream) {
  hipLaunchKernelGGL(k_drain_end, dim3(1), dim3(1), 0, (hipStream_t)stream, p);
  return hipGetLastError();
}

int cg_launch_hostops(const GParams& p, int32_t time, int32_t op_begin, int32_t op_count, void* stream) {
  hipLaunchKernelGGL(k_hostops, dim3(1), dim3(kThreads), 0, (hipStream_t)stream, p, time, op_begin, op_count);
  return hipGetLastError();
}

__global__ void k_sg_begin(GParams p) {
  fold_draw(p.sc);
  p.sc->sg_first = 0x7fffffff;
  p.sc->sg_frozen = p.sc->status;
}

int cg_launch_sendgroup(const GParams& p, int32_t time, int32_t op_begin, int32_t op_count, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const unsigned g = (unsigned)((op_count + kGThreads - 1) / kGThreads);
  hipLaunchKernelGGL(k_sg_begin, dim3(1), dim3(1), 0, s, p);
  hipLaunchKernelGGL(k_sg_check, dim3(g), dim3(kGThreads), 0, s, p, op_begin, op_count);
  hipLaunchKernelGGL(k_sg_apply, dim3(g), dim3(kGThreads), 0, s, p, time, op_begin, op_count);
  return hipGetLastError();
}

int cg_launch_part_pick(const GParams& p, int32_t t, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  if ((e = hipMemsetAsync(p.out_n, 0, 4 * sizeof(uint32_t), s))) return e;
  if (p.blk_hi > p.blk_lo) launch_pick(p, dim3(p.blk_hi - p.blk_lo), t, s);
  return hipGetLastError();
}

int cg_launch_part_receive(const GParams& p, int32_t t, const PDel* in, int32_t n_in, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const unsigned g = (unsigned)((n_in + kGThreads - 1) / kGThreads);
  if (n_in > 0) hipLaunchKernelGGL(k_part_apply, dim3(g), dim3(kGThreads), 0, s, p, t, in, n_in);
  if (p.blk_hi > p.blk_lo)
    hipLaunchKernelGGL(k_marker<false>, dim3(p.blk_hi - p.blk_lo), dim3(kGThreads), 0, s, p, t);
  if (n_in > 0) hipLaunchKernelGGL(k_marker<true>, dim3(g), dim3(kGThreads), 0, s, p, t);
  return hipGetLastError();
}

int cg_launch_part_tally(const GParams& p, int32_t step, const int2* rep, int32_t n_rep, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n_rep > 0) hipLaunchKernelGGL(k_part_trig, dim3((n_rep + kGThreads - 1) / kGThreads), dim3(kGThreads), 0, s, p, rep, n_rep);
  if (p.blk_hi > p.blk_lo) hipLaunchKernelGGL(k_tally, dim3(p.blk_hi - p.blk_lo), dim3(kGThreads), 0, s, p, step);
  launch_scan(p, 0, 0, 0, s);
  return hipGetLastError();
}

int cg_launch_part_bases(const GParams& p, int64_t trig_before, int64_t trig_all, int64_t send_before,
                         int64_t send_all, const int32_t* s0, int32_t n, unsigned long long* draw0, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_part_bases, dim3(1), dim3(1), 0, s, p, (long long)trig_before, (long long)trig_all,
                     (long long)send_before, (long long)send_all);
  if (n > 0) hipLaunchKernelGGL(k_part_draws, dim3((n + kGThreads - 1) / kGThreads), dim3(kGThreads), 0, s, p, s0, n, draw0);
  return hipGetLastError();
}

int cg_launch_part_push(const GParams& p, int32_t t, int32_t step, const long long* replies, int32_t n, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n > 0) hipLaunchKernelGGL(k_part_rdraw, dim3((n + kGThreads - 1) / kGThreads), dim3(kGThreads), 0, s, p, replies, n);
  launch_push(p, t, step, s);
  return hipGetLastError();
}

// ---- device exchange steps (the collectives run between them on the same stream) ----
static unsigned bk_grid(const GParams& p) {
  const int64_t m = (int64_t)p.bk_world * p.bk_cap;
  return (unsigned)((m + kGThreads - 1) / kGThreads);
}

int cg_launch_part_dev_seal(const GParams& p, void* stream) {
  hipLaunchKernelGGL(k_bk_seal, dim3(1), dim3(64), 0, (hipStream_t)stream, p);
  return hipGetLastError();
}

int cg_launch_part_dev_pick(const GParams& p, int32_t t, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  if ((e = hipMemsetAsync(p.out_n, 0, 4 * sizeof(uint32_t), s))) return e;
  if (p.blk_hi > p.blk_lo) launch_pick(p, dim3(p.blk_hi - p.blk_lo), t, s);
  return cg_launch_part_dev_seal(p, stream);
}

int cg_launch_part_dev_receive(const GParams& p, int32_t t, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const unsigned g = bk_grid(p);
  hipLaunchKernelGGL(k_bk_apply, dim3(g), dim3(kGThreads), 0, s, p, t);
  if (p.blk_hi > p.blk_lo)
    hipLaunchKernelGGL(k_marker<false>, dim3(p.blk_hi - p.blk_lo), dim3(kGThreads), 0, s, p, t);
  hipLaunchKernelGGL(k_marker<true>, dim3(g), dim3(kGThreads), 0, s, p, t);  // (blocks past out_n[1] return)
  return cg_launch_part_dev_seal(p, stream);
}

int cg_launch_part_dev_tally(const GParams& p, int32_t step, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_bk_trig, dim3(bk_grid(p)), dim3(kGThreads), 0, s, p);
  if (p.blk_hi > p.blk_lo) hipLaunchKernelGGL(k_tally, dim3(p.blk_hi - p.blk_lo), dim3(kGThreads), 0, s, p, step);
  launch_scan(p, 0, 0, 0, s);
  hipLaunchKernelGGL(k_bk_totals, dim3(1), dim3(1), 0, s, p);
  return hipGetLastError();
}

int cg_launch_part_dev_bases(const GParams& p, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_bk_bases, dim3(1), dim3(1), 0, s, p);
  hipLaunchKernelGGL(k_bk_draws, dim3(bk_grid(p)), dim3(kGThreads), 0, s, p);
  return hipGetLastError();
}

int cg_launch_part_dev_push(const GParams& p, int32_t t, int32_t step, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_bk_rdraw, dim3(bk_grid(p)), dim3(kGThreads), 0, s, p);
  launch_push(p, t, step, s);
  return hipGetLastError();
}

int cg_launch_finish(const GParams& p, int32_t n_sids, unsigned long long* out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int64_t m = (int64_t)n_sids * (p.part_hi - p.part_lo);
  const int g = m ? (grid_for(m) < 8192 ? grid_for(m) : 8192) : 1;
  hipLaunchKernelGGL(k_finish, dim3(g), dim3(kThreads), 0, s, p, n_sids, out);
  return hipGetLastError();
}

int cg_launch_checks(const GParams& p, int32_t n_sids, unsigned long long* out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_checks_state, dim3(1024), dim3(kThreads), 0, s, p, out);
  if (n_sids > 0)
    hipLaunchKernelGGL(k_checks_snap, dim3(64, n_sids < 65535 ? n_sids : 65535), dim3(kThreads), 0, s, p, n_sids, out);
  return hipGetLastError();
}

}  // namespace clsnap
