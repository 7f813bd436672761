// cg_kernels.hip -- gfx950 kernels of the graph engine: one reference simulation over a
// large topology, state in HBM, one tick = a short sequence of grid-wide phases.
//
// Reference semantics restated per phase (paths relative to /root/reference/chandy_lamport):
//   k_pick     Tick (sim.go:71-95): time++, every sender scans its out-links in dest
//              order and pops the first due head (at most one per sender, :90).  Picks
//              from tick-start state equal the reference's sequential picks: a push made
//              during tick t is due at >= t+1 and never changes a non-empty queue's head.
//              Tokens are applied at once (HandleToken node.go:174-185 is commutative for
//              the token count; recording is the channel cursor tokcnt); markers are
//              staged for k_marker.
//   k_marker   HandleMarker (node.go:149-171): the first marker of snapshot s at node v
//              is the one from the lowest-ranked sender in the earliest tick (atomicMin on
//              the creation key W); it creates the local snapshot (CreateLocalSnapshot
//              node.go:58-84) and triggers the broadcast; later markers close their
//              channel.  Completion (node.go:165-168, sim.go:126-131) is the pending
//              accumulator reaching exactly kBig.
//   k_expand   The per-in-link part of CreateLocalSnapshot: recording cursors begin at
//              the channel's delivered-token count AT the creating delivery, i.e. tokens
//              delivered in the same tick by lower-ranked senders are before it and those
//              of higher-ranked senders after it; the recorded node tokens likewise.
//   k_tally    } SendToNeighbors (node.go:97-109) draws one delay per out-link in the
//   k_scan     } reference's global draw order: triggering senders in rank order, then
//   k_push     } the next step's sends in rank order; a two-level exclusive scan over
//              node ranks gives every broadcast/send its draw index.  Each node then
//              pushes onto its own out-channels (broadcasts in creating-sender order,
//              then its send), so FIFO order is the reference's Queue.Push order
//              (queue.go:18-20).
//   k_hostops  ProcessEvent for host events (sim.go:58-68, SendTokens node.go:112-131,
//              StartSnapshot sim.go:105-123 / node.go:198-212), in program order.
#include <hip/hip_runtime.h>

#include "cg_engine.h"

namespace clsnap {
namespace {

constexpr int kThreads = 256;

__device__ inline uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

__device__ inline uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Wave-aggregated append: one atomic per wave, slots in lane order.
__device__ inline int wave_append(int32_t* counter, bool pred) {
  const uint64_t m = __ballot(pred);
  if (m == 0) return -1;
  const int leader = __ffsll((unsigned long long)m) - 1;
  int base = 0;
  if ((int)lane_id() == leader) base = atomicAdd(counter, (int)__popcll(m));
  base = __shfl(base, leader);
  return pred ? base + (int)lanes_below(m) : -1;
}

__device__ inline unsigned long long wave_sum(unsigned long long x) {
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

// Add a per-lane count to a device counter, one atomic per wave.
__device__ inline void wave_count(unsigned long long* dst, unsigned long long x) {
  x = wave_sum(x);
  if (lane_id() == 0 && x) atomicAdd(dst, x);
}

__device__ inline void set_status(GScal* sc, int32_t code) { atomicCAS(&sc->status, 0, code); }

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

// Queue.Push (queue.go:18-20) onto out-channel j of node v.
__device__ inline void push_entry(const GParams& p, int32_t c, int32_t j, uint64_t& mask, uint32_t payload,
                                  uint32_t rt, unsigned long long& pushes) {
  const uint32_t hc = p.hc[c];
  const uint32_t head = hc & 0xffffu, cnt = hc >> 16, cap = 1u << p.cap_log2;
  if (cnt >= cap) {
    set_status(p.sc, ST_FIFO_OVERFLOW);
    return;
  }
  p.fifo[((size_t)c << p.cap_log2) + ((head + cnt) & (cap - 1))] = ((uint64_t)rt << 32) | payload;
  p.hc[c] = head | ((cnt + 1) << 16);
  mask |= 1ull << j;
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

__device__ inline void complete_node(const GParams& p, int32_t sid, int32_t t, unsigned long long& completed) {
  const int d = atomicAdd(&p.done[sid], 1) + 1;  // NotifyCompletedSnapshot, sim.go:126-131
  if (d == p.n) {
    p.ctick[sid] = t;
    ++completed;
  }
}

// ---------------------------------------------------------------------------
// reset
// ---------------------------------------------------------------------------
__global__ void k_reset_nodes(GParams p, const int32_t* init_tok) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v < p.n) {
    p.tokens[v] = init_tok[v];
    p.mask[v] = 0;
    p.pick[v] = -1;
    p.trig[v] = 0;
    p.crn[v] = 0;
  }
  if (v < p.s_cap) {
    p.done[v] = 0;
    p.ctick[v] = -1;
  }
}

// ---------------------------------------------------------------------------
// tick phase A: pick + deliver
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kThreads) k_pick(GParams p, int32_t t) {
  if (p.sc->status) return;
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s == 0) p.sc->time = t;  // time++ (sim.go:72)
  unsigned long long peeks = 0, ptok = 0, pmk = 0;
  bool marker = false;
  if (s < p.n) {
    uint64_t m = p.mask[s];
    if (m) {
      const uint64_t m0 = m;
      const int32_t base = p.out_off[s];
      const uint32_t capm = (1u << p.cap_log2) - 1;
      while (m) {
        const int j = __builtin_ctzll(m);
        m &= m - 1;
        const int32_t c = base + j;
        const uint32_t hc = p.hc[c];
        const uint32_t head = hc & 0xffffu;
        const uint64_t e = p.fifo[((size_t)c << p.cap_log2) + head];
        ++peeks;  // Queue.Peek, sim.go:83
        if ((uint32_t)(e >> 32) > (uint32_t)t) continue;
        const uint32_t cnt = (hc >> 16) - 1;
        p.hc[c] = ((head + 1) & capm) | (cnt << 16);
        if (cnt == 0) p.mask[s] = m0 & ~(1ull << j);
        p.pick[s] = (t << 6) | j;
        const int32_t v = p.ch_dst[c], k = p.ch_inpos[c];
        const uint32_t pay = (uint32_t)e;
        if (pay & kGMarker) {
          const uint32_t sid = pay & kGPayload;
          atomicMin((unsigned long long*)&p.W[(size_t)sid * p.n + v], ((unsigned long long)t << 32) | (uint32_t)s);
          marker = true;
          ++pmk;
        } else {
          atomicAdd(&p.tokens[v], (int32_t)pay);  // HandleToken node.go:175
          const uint32_t tc = p.tokcnt[k];
          if (p.hist) {
            if (tc < (uint32_t)p.hist) p.histv[(size_t)k * p.hist + tc] = pay;
            else set_status(p.sc, kGStatusHistOverflow);
          }
          p.tokcnt[k] = tc + 1;
          ++ptok;
        }
        p.deliv[k] = ((uint64_t)t << 32) | pay;
        break;
      }
    }
  }
  const int slot = wave_append(&p.sc->mlist_n, marker);
  if (marker) p.mlist[slot] = s;
  wave_count(&p.sc->peek, peeks);
  wave_count(&p.sc->pop_tok, ptok);
  wave_count(&p.sc->pop_mk, pmk);
}

// ---------------------------------------------------------------------------
// tick phase B: markers
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kThreads) k_marker(GParams p, int32_t t) {
  if (p.sc->status) return;
  const int nm = p.sc->mlist_n;
  unsigned long long recorded = 0, completed = 0;
  const int stride = gridDim.x * blockDim.x;
  const int i0 = blockIdx.x * blockDim.x + threadIdx.x;
  // uniform trip count per wave so wave_append sees every lane
  const int trips = (nm + stride - 1) / stride;
  for (int it = 0; it < trips; ++it) {
    const int i = i0 + it * stride;
    bool creator = false;
    int32_t s0 = 0;
    if (i < nm) {
      s0 = p.mlist[i];
      const int32_t c = p.out_off[s0] + (p.pick[s0] & 63);
      const int32_t v = p.ch_dst[c], k = p.ch_inpos[c];
      const int32_t sid = (int32_t)((uint32_t)p.deliv[k] & kGPayload);
      const size_t sv = (size_t)sid * p.n + v;
      const uint64_t key = p.W[sv];
      const int32_t indeg = p.in_off[v + 1] - p.in_off[v];
      if (key == (((uint64_t)t << 32) | (uint32_t)s0)) {
        // first marker: CreateLocalSnapshot(src) + SendToNeighbors (node.go:153-156)
        creator = true;
        p.trig[s0] = p.out_off[v + 1] - p.out_off[v];
        const int slot = atomicAdd(&p.crn[v], 1);
        p.cre[p.in_off[v] + slot] = ((uint64_t)(uint32_t)s0 << 32) | (uint32_t)sid;
        const int add = kBig + indeg - 1;
        if (atomicAdd(&p.cnt[sv], add) + add == kBig) complete_node(p, sid, t, completed);
      } else {
        // later marker: stop recording the channel (node.go:158-160)
        if ((key >> 32) != (uint64_t)t) {  // created in an earlier tick: cursors exist
          const uint32_t e = p.tokcnt[k];
          uint32_t* r = (uint32_t*)&p.rec[(size_t)sid * p.e + k];
          recorded += e - r[0];
          r[1] = e;
        }  // else created this tick by a lower-ranked sender: k_expand closes it
        if (atomicAdd(&p.cnt[sv], -1) - 1 == kBig) complete_node(p, sid, t, completed);
      }
    }
    const int slot = wave_append(&p.sc->xl_n, creator);
    if (creator) p.xl[slot] = s0;
  }
  wave_count(&p.sc->recorded, recorded);
  wave_count(&p.sc->completed, completed);
}

// ---------------------------------------------------------------------------
// tick phase C: expand the local snapshots created this tick over their in-links.
// `L` lanes cooperate on one creation (L = power of two <= 64).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kThreads) k_expand(GParams p, int32_t t, int32_t L) {
  if (p.sc->status) return;
  const int nx = p.sc->xl_n;
  const int gtid = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = gtid & (L - 1);
  const int groups = gridDim.x * blockDim.x / L;
  const int trips = (nx + groups - 1) / groups;
  for (int it = 0; it < trips; ++it) {
    const int i = gtid / L + it * groups;
    int tsum = 0;
    int32_t v = 0, sid = 0;
    if (i < nx) {
      const int32_t s0 = p.xl[i];
      const int32_t c = p.out_off[s0] + (p.pick[s0] & 63);
      v = p.ch_dst[c];
      const int32_t karr = p.ch_inpos[c];
      sid = (int32_t)((uint32_t)p.deliv[karr] & kGPayload);
      const int32_t lo = p.in_off[v], hi = p.in_off[v + 1];
      uint64_t* rec = p.rec + (size_t)sid * p.e;
      for (int32_t k = lo + lane; k < hi; k += L) {
        uint32_t b = p.tokcnt[k];
        const uint64_t dv = p.deliv[k];
        bool closed = k == karr;  // the arriving channel does not record (node.go:66-69)
        if ((dv >> 32) == (uint64_t)t && p.in_src[k] > s0) {
          const uint32_t pay = (uint32_t)dv;
          if (!(pay & kGMarker)) {
            b -= 1;  // delivered after the creating marker: recorded
            tsum += (int)pay;
          } else if ((int32_t)(pay & kGPayload) == sid) {
            closed = true;  // its own marker arrives later in the same tick
          }
        }
        rec[k] = (uint64_t)b | ((uint64_t)(closed ? b : kOpen) << 32);
      }
    }
    for (int o = L >> 1; o > 0; o >>= 1) tsum += __shfl_xor(tsum, o, L);
    if (i < nx && lane == 0) p.stok[(size_t)sid * p.n + v] = p.tokens[v] - tsum;
  }
}

// ---------------------------------------------------------------------------
// block exclusive scan of (a, b) pairs over blockDim.x threads (multiple of 64)
// ---------------------------------------------------------------------------
__device__ inline void block_exclusive_scan2(long long& a, long long& b, long long& tot_a, long long& tot_b,
                                             long long* sh /* [2 * 16] */) {
  const int lane = (int)lane_id(), w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  long long ia = a, ib = b;
  for (int o = 1; o < 64; o <<= 1) {
    const long long xa = __shfl_up(ia, o), xb = __shfl_up(ib, o);
    if (lane >= o) {
      ia += xa;
      ib += xb;
    }
  }
  if (lane == 63) {
    sh[2 * w] = ia;
    sh[2 * w + 1] = ib;
  }
  __syncthreads();
  long long pa = 0, pb = 0;
  tot_a = tot_b = 0;
  for (int k = 0; k < nw; ++k) {
    if (k < w) {
      pa += sh[2 * k];
      pb += sh[2 * k + 1];
    }
    tot_a += sh[2 * k];
    tot_b += sh[2 * k + 1];
  }
  __syncthreads();
  a = pa + ia - a;
  b = pb + ib - b;
}

// ---------------------------------------------------------------------------
// tick phase D: tally triggers (this tick) and traffic sends (step `step`) per block
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kThreads) k_tally(GParams p, int32_t step) {
  if (p.sc->status) return;
  __shared__ long long sh[32];
  const int base = blockIdx.x * kTallyBlock + threadIdx.x * 4;
  int tr[4], se[4];
  long long a = 0, b = 0;
  for (int q = 0; q < 4; ++q) {
    const int v = base + q;
    tr[q] = se[q] = 0;
    if (v < p.n) {
      tr[q] = p.trig[v];
      if (tr[q]) p.trig[v] = 0;
      int32_t j;
      se[q] = traffic_send(p, step, v, p.out_off[v + 1] - p.out_off[v], p.tokens[v], &j) ? 1 : 0;
    }
    a += tr[q];
    b += se[q];
  }
  long long ta, tb;
  block_exclusive_scan2(a, b, ta, tb, sh);
  for (int q = 0; q < 4; ++q) {
    const int v = base + q;
    if (tr[q]) p.ltrig[v] = (int32_t)a;
    if (se[q]) p.lsend[v] = (int32_t)b;
    a += tr[q];
    b += se[q];
  }
  if (threadIdx.x == 0) {
    p.bsum[2 * blockIdx.x] = ta;
    p.bsum[2 * blockIdx.x + 1] = tb;
  }
}

// phase E: exclusive scan of the block sums (one workgroup), draw bases
__global__ void __launch_bounds__(1024) k_scan(GParams p) {
  if (p.sc->status) return;
  __shared__ long long sh[32];
  long long carry_a = 0, carry_b = 0;
  for (int c0 = 0; c0 < p.n_blocks; c0 += blockDim.x) {
    const int i = c0 + threadIdx.x;
    long long a = i < p.n_blocks ? p.bsum[2 * i] : 0, b = i < p.n_blocks ? p.bsum[2 * i + 1] : 0;
    long long ta, tb;
    block_exclusive_scan2(a, b, ta, tb, sh);
    if (i < p.n_blocks) {
      p.bsum[2 * i] = carry_a + a;
      p.bsum[2 * i + 1] = carry_b + b;
    }
    carry_a += ta;
    carry_b += tb;
  }
  if (threadIdx.x == 0) {
    const unsigned long long d = p.sc->draw;
    p.sc->base_trig = d;
    p.sc->base_send = d + (unsigned long long)carry_a;
    p.sc->draw = d + (unsigned long long)(carry_a + carry_b);
  }
}

// phase F: every node pushes onto its own out-channels -- the broadcasts of the local
// snapshots created at it this tick (in creating-sender order), then its traffic send.
__global__ void __launch_bounds__(kThreads) k_push(GParams p, int32_t t, int32_t step) {
  if (p.sc->status) return;
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long pushes = 0, peeks = 0;
  if (v < p.n) {
    const int32_t ob = p.out_off[v], od = p.out_off[v + 1] - ob;
    uint64_t mask = p.mask[v];
    const uint64_t mask0 = mask;
    const int ncre = p.crn[v];
    if (ncre) {
      p.crn[v] = 0;
      const int32_t lo = p.in_off[v];
      uint64_t prev = 0;
      for (int r = 0; r < ncre; ++r) {
        uint64_t best = ~0ull;
        for (int i = 0; i < ncre; ++i) {
          const uint64_t x = p.cre[lo + i];
          if ((r == 0 || x > prev) && x < best) best = x;
        }
        prev = best;
        const int32_t s0 = (int32_t)(best >> 32);
        const uint32_t sid = (uint32_t)best;
        if (r == 0 && s0 < v) {
          // The reference delivers s0's marker before v's own turn in this tick, so v's
          // scan peeks the queues the broadcast made non-empty (sim.go:82-84).
          const int pk = p.pick[v];
          const int pj = (pk >> 6) == t ? (pk & 63) : 64;
          for (int j = 0; j < od && j < pj; ++j)
            if (!((mask0 >> j) & 1)) ++peeks;
        }
        const unsigned long long draw0 = p.sc->base_trig + (unsigned long long)p.bsum[2 * (s0 / kTallyBlock)] +
                                         (unsigned long long)p.ltrig[s0];
        for (int j = 0; j < od; ++j)
          push_entry(p, ob + j, j, mask, kGMarker | sid, receive_time(p, draw0 + j, t), pushes);
      }
    }
    int32_t j;
    const int32_t tok = p.tokens[v];
    if (traffic_send(p, step, v, od, tok, &j)) {
      // SendTokens(v, out-link j, 1): node.go:112-131
      const unsigned long long draw = p.sc->base_send + (unsigned long long)p.bsum[2 * (v / kTallyBlock) + 1] +
                                      (unsigned long long)p.lsend[v];
      p.tokens[v] = tok - 1;
      push_entry(p, ob + j, j, mask, 1u, receive_time(p, draw, t), pushes);
    }
    if (mask != mask0) p.mask[v] = mask;
  }
  wave_count(&p.sc->push, pushes);
  wave_count(&p.sc->peek, peeks);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    p.sc->mlist_n = 0;
    p.sc->xl_n = 0;
  }
}

// ---------------------------------------------------------------------------
// host events of one step, in program order (one workgroup)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kThreads) k_hostops(GParams p, int32_t time, int32_t ob, int32_t oc) {
  __shared__ int s_stop;
  for (int i = 0; i < oc; ++i) {
    const GOp op = p.ops[ob + i];
    if (threadIdx.x == 0) s_stop = p.sc->status != 0;
    __syncthreads();
    if (s_stop) return;
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
            if (p.ch_dst[obv + mid] < op.b) lo = mid + 1;
            else hi = mid;
          }
          if (op.b < 0 || lo >= od || p.ch_dst[obv + lo] != op.b) {
            set_status(p.sc, ST_FATAL_UNKNOWN_DEST);
          } else {
            uint64_t mask = p.mask[v];
            unsigned long long pushes = 0;
            const unsigned long long d = p.sc->draw++;
            push_entry(p, obv + lo, lo, mask, (uint32_t)op.n, receive_time(p, d, time), pushes);
            p.mask[v] = mask;
            p.sc->push += pushes;
          }
        }
      }
    } else {
      // StartSnapshot (sim.go:105-123 -> node.go:198-212): CreateLocalSnapshot("") records
      // every in-link, then SendToNeighbors
      const int32_t sid = op.b;
      const int32_t lo = p.in_off[v], hi = p.in_off[v + 1];
      uint64_t* rec = p.rec + (size_t)sid * p.e;
      for (int32_t k = lo + (int32_t)threadIdx.x; k < hi; k += blockDim.x)
        rec[k] = (uint64_t)p.tokcnt[k] | ((uint64_t)kOpen << 32);
      if (threadIdx.x == 0) {
        const size_t sv = (size_t)sid * p.n + v;
        p.W[sv] = ((uint64_t)(uint32_t)time << 32) | 0xffffffffull;
        p.stok[sv] = p.tokens[v];
        atomicAdd(&p.cnt[sv], kBig + (hi - lo));
        uint64_t mask = p.mask[v];
        unsigned long long pushes = 0;
        const unsigned long long d = p.sc->draw;
        for (int j = 0; j < od; ++j)
          push_entry(p, obv + j, j, mask, kGMarker | (uint32_t)sid, receive_time(p, d + j, time), pushes);
        p.sc->draw = d + od;
        p.mask[v] = mask;
        p.sc->push += pushes;
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// results
// ---------------------------------------------------------------------------
// Recorded copies of channels still recording at the end (HandleToken appended them).
__global__ void k_finish(GParams p, int32_t n_sids, unsigned long long* out) {
  const size_t total = (size_t)n_sids * p.n;
  unsigned long long rec = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int32_t sid = (int32_t)(i / p.n), v = (int32_t)(i % p.n);
    if (p.W[i] == ~0ull || p.cnt[i] == kBig) continue;
    const uint64_t* r = p.rec + (size_t)sid * p.e;
    for (int32_t k = p.in_off[v]; k < p.in_off[v + 1]; ++k) {
      const uint64_t x = r[k];
      if ((uint32_t)(x >> 32) == kOpen) rec += p.tokcnt[k] - (uint32_t)x;
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
  for (size_t v = gt; v < (size_t)p.n; v += gs) fin += (unsigned long long)(long long)p.tokens[v];
  const uint32_t capm = (1u << p.cap_log2) - 1;
  for (size_t c = gt; c < (size_t)p.e; c += gs) {
    const uint32_t hc = p.hc[c];
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
    const int32_t* stok = p.stok + (size_t)sid * p.n;
    for (size_t v = gt; v < (size_t)p.n; v += gs) {
      const int32_t st = stok[v];
      dig += mix64(cg_hash(0x5107ull, (uint64_t)sid, (uint64_t)v) ^ (uint64_t)(uint32_t)st);
      cut += (unsigned long long)(long long)st;
    }
    const uint64_t* rec = p.rec + (size_t)sid * p.e;
    for (size_t c = gt; c < (size_t)p.e; c += gs) {
      const int32_t k = p.ch_inpos[c];
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
  if ((e = hipMemsetAsync(p.hc, 0, (size_t)p.e * sizeof(uint32_t), s))) return e;
  if ((e = hipMemsetAsync(p.tokcnt, 0, (size_t)p.e * sizeof(uint32_t), s))) return e;
  if ((e = hipMemsetAsync(p.deliv, 0, (size_t)p.e * sizeof(uint64_t), s))) return e;
  if ((e = hipMemsetAsync(p.W, 0xff, (size_t)p.s_cap * p.n * sizeof(uint64_t), s))) return e;
  if ((e = hipMemsetAsync(p.cnt, 0, (size_t)p.s_cap * p.n * sizeof(int32_t), s))) return e;
  if ((e = hipMemsetAsync(p.sc, 0, sizeof(GScal), s))) return e;
  const int64_t m = p.n > p.s_cap ? p.n : p.s_cap;
  hipLaunchKernelGGL(k_reset_nodes, dim3(grid_for(m)), dim3(kThreads), 0, s, p, init_tok);
  return hipGetLastError();
}

int cg_launch_sends(const GParams& p, int32_t t, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_tally, dim3(p.n_blocks), dim3(kThreads), 0, s, p, t);
  hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, s, p);
  hipLaunchKernelGGL(k_push, dim3(grid_for(p.n)), dim3(kThreads), 0, s, p, t, t);
  return hipGetLastError();
}

int cg_launch_tick(const GParams& p, int32_t t, int32_t lanes_per_creation, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int list_grid = grid_for(p.n) < 2048 ? grid_for(p.n) : 2048;
  hipLaunchKernelGGL(k_pick, dim3(grid_for(p.n)), dim3(kThreads), 0, s, p, t);
  hipLaunchKernelGGL(k_marker, dim3(list_grid), dim3(kThreads), 0, s, p, t);
  const int xg = grid_for((int64_t)p.n * lanes_per_creation);
  hipLaunchKernelGGL(k_expand, dim3(xg < 4096 ? xg : 4096), dim3(kThreads), 0, s, p, t, lanes_per_creation);
  hipLaunchKernelGGL(k_tally, dim3(p.n_blocks), dim3(kThreads), 0, s, p, t);
  hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, s, p);
  hipLaunchKernelGGL(k_push, dim3(grid_for(p.n)), dim3(kThreads), 0, s, p, t, t);
  return hipGetLastError();
}

int cg_launch_hostops(const GParams& p, int32_t time, int32_t op_begin, int32_t op_count, void* stream) {
  hipLaunchKernelGGL(k_hostops, dim3(1), dim3(kThreads), 0, (hipStream_t)stream, p, time, op_begin, op_count);
  return hipGetLastError();
}

int cg_launch_finish(const GParams& p, int32_t n_sids, unsigned long long* out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int64_t m = (int64_t)n_sids * p.n;
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
