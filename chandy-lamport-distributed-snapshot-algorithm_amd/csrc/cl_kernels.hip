// cl_kernels.hip -- gfx950 kernels of the Chandy-Lamport batch engine.
//
// cl_exec_kernel runs the event program (send / snapshot / tick / drain) for 64
// independent simulator instances per wave, one instance per lane.  Each instance's
// mutable state (channel FIFOs, node tokens, per-snapshot bookkeeping) lives in LDS for
// the whole launch, laid out lane-column-major (word k of lane l at lds[k*64 + l]) so
// every data-dependent per-lane access is bank-conflict free.  The topology and the
// program are uniform across lanes and are read through the scalar cache.  Only the
// delay schedule (1 B per draw), the snapshot outputs and the saved state touch HBM.
//
// Semantics restated (paths relative to /root/reference/chandy_lamport):
//   tick()          sim.go:71-95   senders in rank order, out-links in dest order,
//                                  head-of-line only, at most one delivery per sender
//   push()          node.go:107,126-130 + sim.go:100-102 (receiveTime = time+1+delay)
//   handle_marker() node.go:149-171, CreateLocalSnapshot node.go:58-84
//   token delivery  node.go:174-185 (recording kept as per-channel cursors)
//   OP_SEND         node.go:112-131 (fatal checks in the reference's order)
//   OP_SNAP         sim.go:105-123, node.go:198-212
//   OP_DRAIN        test_common.go:123-137
#include <hip/hip_runtime.h>

#include "cl_engine.h"

// Diagnostic ablations (never set in the shipped build): CLSNAP_ABL_NOSTORE drops the
// snapshot-output stores inside the tick loop, CLSNAP_ABL_NODELAYLOAD replaces the delay
// schedule with zeros.  Outputs are wrong in those builds; only timing is meaningful.
#ifndef CLSNAP_ABL_NOSTORE
#define CLSNAP_ABL_NOSTORE 0
#endif
#ifndef CLSNAP_ABL_NODELAYLOAD
#define CLSNAP_ABL_NODELAYLOAD 0
#endif

namespace clsnap {
namespace {

// Uniform inputs: parameters, topology and delay schedule.
struct Ctx {
  const ExecParams& p;
  TopoView t;
  const uint8_t* __restrict__ sched;
};

struct Lane {
  uint32_t* L;  // lds + lane
  int64_t inst;
  int32_t time, dptr, status, ndone;
  uint32_t peek, pop_tok, pop_mk, push;
  bool alive;
  // Delay window: draws [wbase, wbase+16) in d0..d3, the next 16 in n0..n3 (in flight).
  int32_t wbase;
  uint32_t d0, d1, d2, d3, n0, n1, n2, n3;
};

// Load the 16 draws starting at byte offset k of this instance's schedule row.
__device__ __forceinline__ uint4 load_window(const Ctx& x, const Lane& ln, int32_t k) {
  if (CLSNAP_ABL_NODELAYLOAD || k >= x.p.sched_row) return make_uint4(0, 0, 0, 0);
  return *reinterpret_cast<const uint4*>(x.sched + ln.inst * x.p.sched_row + k);
}

__device__ __forceinline__ void open_window(const Ctx& x, Lane& ln) {
  ln.wbase = ln.dptr & ~15;
  const uint4 a = load_window(x, ln, ln.wbase);
  const uint4 b = load_window(x, ln, ln.wbase + 16);
  ln.d0 = a.x; ln.d1 = a.y; ln.d2 = a.z; ln.d3 = a.w;
  ln.n0 = b.x; ln.n1 = b.y; ln.n2 = b.z; ln.n3 = b.w;
  for (int32_t k = ln.wbase; k < ln.dptr; ++k) {  // resume mid-window
    ln.d0 = __builtin_amdgcn_alignbit(ln.d1, ln.d0, 8);
    ln.d1 = __builtin_amdgcn_alignbit(ln.d2, ln.d1, 8);
    ln.d2 = __builtin_amdgcn_alignbit(ln.d3, ln.d2, 8);
    ln.d3 >>= 8;
  }
}

// Next delay draw (replaces rand.Intn(maxDelay), sim.go:101); caller checked dptr < draws.
// The current window is consumed from its low byte and shifted down (v_alignbit), so no
// runtime-indexed register selection is needed.
__device__ __forceinline__ uint32_t next_delay(const Ctx& x, Lane& ln) {
  const uint32_t d = ln.d0 & 0xffu;
  ln.d0 = __builtin_amdgcn_alignbit(ln.d1, ln.d0, 8);
  ln.d1 = __builtin_amdgcn_alignbit(ln.d2, ln.d1, 8);
  ln.d2 = __builtin_amdgcn_alignbit(ln.d3, ln.d2, 8);
  ln.d3 >>= 8;
  ln.dptr++;
  if ((ln.dptr & 15) == 0) {  // slide: the prefetched window becomes current, prefetch the next one
    ln.wbase += 16;
    ln.d0 = ln.n0; ln.d1 = ln.n1; ln.d2 = ln.n2; ln.d3 = ln.n3;
    const uint4 b = load_window(x, ln, ln.wbase + 16);
    ln.n0 = b.x; ln.n1 = b.y; ln.n2 = b.z; ln.n3 = b.w;
  }
  return d;
}

#define LW(k) (ln.L[(uint32_t)(k) << 6])

__device__ __forceinline__ void fail(Lane& ln, int32_t st) {
  ln.status = st;
  ln.alive = false;
}

// Queue.Push (queue.go:18-20) with the receive time drawn at push (sim.go:100-102).
__device__ __forceinline__ void push(const Ctx& x, Lane& ln, int32_t c, uint32_t payload) {
  if (!ln.alive) return;
  const ExecParams& p = x.p;
  const Layout& lay = p.lay;
  const uint32_t chw = LW(lay.w_chw + c);
  const uint32_t cnt = (chw >> 8) & 0xffu;
  if (cnt >= (uint32_t)kMaxQueued) { fail(ln, ST_FIFO_OVERFLOW); return; }
  if (ln.dptr >= p.draws) { fail(ln, ST_DELAY_EXHAUSTED); return; }
  const uint32_t delay = next_delay(x, ln);
  const uint32_t e = payload | ((uint32_t)(ln.time + 1 + (int32_t)delay) << 16);
  const uint32_t cap = 1u << lay.cap_log2;
  if (cnt < cap) {
    LW(lay.w_fifo + ((uint32_t)c << lay.cap_log2) + ((chw + cnt) & (cap - 1))) = e;
  } else {
    // LDS ring full: the channel's younger packets spill to an HBM ring.
    if (lay.ocap_log2 < 0 || cnt - cap >= (1u << lay.ocap_log2)) { fail(ln, ST_FIFO_OVERFLOW); return; }
    const uint32_t om = (1u << lay.ocap_log2) - 1;
    const uint32_t h = p.ovh[(int64_t)c * p.stride + ln.inst];
    p.ovf[(((int64_t)c << lay.ocap_log2) + ((h + cnt - cap) & om)) * p.stride + ln.inst] = e;
  }
  LW(lay.w_chw + c) = chw + kCountOne;
  ln.push++;
}

// SendToNeighbors (node.go:97-109): one draw per out-link, dest order.
__device__ __forceinline__ void broadcast_marker(const Ctx& x, Lane& ln, int32_t w, int32_t sid) {
  const int32_t e0 = x.t.out_off[w], e1 = x.t.out_off[w + 1];
  for (int32_t c = e0; c < e1; ++c) push(x, ln, c, kMarkerBit | (uint32_t)sid);
}

// CreateLocalSnapshot (node.go:58-84): record tokens, open every in-channel except the
// one the first marker arrived on (arrive = -1 for the initiator).  A channel's
// recording is the half-open cursor interval [begin, end) over the tokens delivered on
// it; end is written when the channel's marker arrives.
__device__ __forceinline__ void create_local(const Ctx& x, Lane& ln, int32_t w, int32_t sid,
                                             int32_t arrive) {
  const ExecParams& p = x.p;
  const Layout& lay = p.lay;
  if (!CLSNAP_ABL_NOSTORE)
    p.snap_tok[((int64_t)sid * p.n_nodes + w) * p.stride + ln.inst] = (int32_t)LW(lay.w_tok + w);
  const int32_t k0 = x.t.in_off[w], k1 = x.t.in_off[w + 1];
  for (int32_t k = k0; k < k1; ++k) {
    const int32_t cc = x.t.in_ch[k];
    const uint32_t td = LW(lay.w_chw + cc) >> 16;
    if (!CLSNAP_ABL_NOSTORE)
      p.snap_rec[((int64_t)sid * p.n_ch + cc) * p.stride + ln.inst] = cc == arrive ? (td | (td << 16)) : td;
  }
}

// NotifyCompletedSnapshot (sim.go:126-131): global completion when all N nodes finished.
__device__ __forceinline__ void node_complete(const ExecParams& p, Lane& ln, int32_t sid) {
  const Layout& lay = p.lay;
  const uint32_t di = lay.w_done + (sid >> 2);
  const uint32_t sh = (sid & 3) * 8;
  const uint32_t dw = LW(di);
  const uint32_t n = ((dw >> sh) & 0xffu) + 1;
  LW(di) = (dw & ~(0xffu << sh)) | (n << sh);
  if (n == (uint32_t)p.n_nodes) {
    if (!CLSNAP_ABL_NOSTORE) p.snap_tick[(int64_t)sid * p.stride + ln.inst] = ln.time;
    ln.ndone++;
  }
}

// HandleMarker (node.go:149-171) at node w, arriving on channel c.
__device__ __forceinline__ void handle_marker(const Ctx& x, Lane& ln, int32_t w, int32_t c,
                                              int32_t sid) {
  const ExecParams& p = x.p;
  const Layout& lay = p.lay;
  const uint32_t st = LW(lay.w_started + w);
  const uint32_t pi = lay.w_pend + w * lay.sp + (sid >> 2);
  const uint32_t sh = (sid & 3) * 8;
  const uint32_t pw = LW(pi);
  int32_t pend;
  if (!((st >> sid) & 1u)) {
    LW(lay.w_started + w) = st | (1u << sid);
    create_local(x, ln, w, sid, c);
    pend = (x.t.in_off[w + 1] - x.t.in_off[w]) - 1;
    broadcast_marker(x, ln, w, sid);
  } else {
    const uint32_t td = LW(lay.w_chw + c) >> 16;
    if (!CLSNAP_ABL_NOSTORE)
      reinterpret_cast<uint16_t*>(p.snap_rec)[2 * (((int64_t)sid * p.n_ch + c) * p.stride + ln.inst) + 1] =
          (uint16_t)td;
    pend = (int32_t)((pw >> sh) & 0xffu) - 1;
  }
  LW(pi) = (pw & ~(0xffu << sh)) | ((uint32_t)pend << sh);
  if (pend == 0) node_complete(p, ln, sid);
}

// Tick (sim.go:71-95).
__device__ __forceinline__ void tick(const Ctx& x, Lane& ln) {
  const ExecParams& p = x.p;
  const Layout& lay = p.lay;
  const uint32_t cap = 1u << lay.cap_log2;
  ln.time++;
  for (int32_t v = 0; v < p.n_nodes; ++v) {
    const int32_t e0 = x.t.out_off[v], e1 = x.t.out_off[v + 1];
    bool done = !ln.alive;
    for (int32_t c = e0; c < e1; ++c) {
      if (done) continue;
      const uint32_t chw = LW(lay.w_chw + c);
      const uint32_t cnt = (chw >> 8) & 0xffu;
      if (!cnt) continue;
      ln.peek++;
      const uint32_t head = chw & 0xffu;
      const uint32_t slot = lay.w_fifo + ((uint32_t)c << lay.cap_log2) + head;
      const uint32_t e = LW(slot);
      if ((int32_t)((e >> 16) & 0x7fffu) > ln.time) continue;
      done = true;
      const bool mk = (e & kMarkerBit) != 0;
      if (cnt > cap) {  // refill the freed slot (the new tail) from the HBM spill ring
        const uint32_t om = (1u << lay.ocap_log2) - 1;
        uint32_t* hp = &p.ovh[(int64_t)c * p.stride + ln.inst];
        const uint32_t h = *hp;
        LW(slot) = p.ovf[(((int64_t)c << lay.ocap_log2) + h) * p.stride + ln.inst];
        *hp = (h + 1) & om;
      }
      LW(lay.w_chw + c) = (chw & 0xffff0000u) + ((cnt - 1) << 8) + ((head + 1) & (cap - 1)) +
                          (mk ? 0u : kTokDelivOne);
      const int32_t w = x.t.ch_dst[c];
      if (mk) {
        ln.pop_mk++;
        handle_marker(x, ln, w, c, (int32_t)(e & 0xffffu));
      } else {
        ln.pop_tok++;
        LW(lay.w_tok + w) += e & 0xffffu;  // HandleToken: tokens += data
      }
    }
  }
}

__global__ __launch_bounds__(64) void cl_exec_kernel(ExecParams p, const int32_t* __restrict__ topo,
                                                     const Op* __restrict__ ops,
                                                     const uint8_t* __restrict__ sched) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const int32_t N = p.n_nodes, C = p.n_ch;
  const Ctx x{p, TopoView{topo, topo + (N + 1), topo + (N + 1) + C, topo + 2 * (N + 1) + C,
                          topo + 2 * (N + 1) + 2 * C},
              sched};
  Lane ln;
  const int lane = threadIdx.x;
  ln.L = lds + lane;
  ln.inst = (int64_t)blockIdx.x * kWave + lane;
  const bool valid = ln.inst < p.n_inst;
  const Layout& lay = p.lay;

  if (p.fresh) {
    for (int32_t k = 0; k < lay.words; ++k) LW(k) = 0u;
    for (int32_t v = 0; v < p.n_nodes; ++v) LW(lay.w_tok + v) = (uint32_t)x.t.init_tok[v];
    ln.time = ln.dptr = ln.status = ln.ndone = 0;
    ln.peek = ln.pop_tok = ln.pop_mk = ln.push = 0;
  } else {
    for (int32_t k = 0; k < lay.words; ++k) LW(k) = p.state[(int64_t)k * p.stride + ln.inst];
    const int32_t* r = p.regs + ln.inst;
    ln.time = r[R_TIME * p.stride];
    ln.dptr = r[R_DRAW * p.stride];
    ln.status = r[R_STATUS * p.stride];
    ln.ndone = r[R_NDONE * p.stride];
    ln.peek = (uint32_t)r[R_PEEK * p.stride];
    ln.pop_tok = (uint32_t)r[R_POP_TOK * p.stride];
    ln.pop_mk = (uint32_t)r[R_POP_MK * p.stride];
    ln.push = (uint32_t)r[R_PUSH * p.stride];
  }
  ln.alive = valid && ln.status == ST_OK;
  if (ln.alive) open_window(x, ln);
  int32_t n_started = p.n_started_before;

  for (int32_t i = p.op_begin; i < p.op_end; ++i) {
    const Op op = ops[i];
    if (op.kind == OP_SEND) {
      // SendTokens: balance check, then link lookup, then push (node.go:113-130)
      if (ln.alive) {
        const int32_t t = (int32_t)LW(lay.w_tok + op.a);
        if (t < op.c) {
          fail(ln, ST_FATAL_INSUFFICIENT);
        } else if (op.b < 0) {
          fail(ln, ST_FATAL_UNKNOWN_DEST);
        } else {
          LW(lay.w_tok + op.a) = (uint32_t)(t - op.c);
          push(x, ln, op.b, (uint32_t)op.c);
        }
      }
    } else if (op.kind == OP_SNAP) {
      // sim.StartSnapshot -> node.StartSnapshot: initiator records every in-channel
      if (ln.alive) {
        const int32_t v = op.a, sid = op.b;
        LW(lay.w_started + v) |= 1u << sid;
        create_local(x, ln, v, sid, -1);
        const uint32_t pi = lay.w_pend + v * lay.sp + (sid >> 2);
        const uint32_t sh = (sid & 3) * 8;
        const uint32_t indeg = (uint32_t)(x.t.in_off[v + 1] - x.t.in_off[v]);
        LW(pi) = (LW(pi) & ~(0xffu << sh)) | (indeg << sh);
        broadcast_marker(x, ln, v, sid);
      }
      n_started++;
    } else if (op.kind == OP_TICK) {
      for (int32_t k = 0; k < op.a; ++k)
        if (ln.alive) tick(x, ln);
    } else if (op.kind == OP_DRAIN) {
      // tick until every started snapshot completed (per instance), then op.b more
      for (int32_t dt = 0;; ++dt) {
        const bool need = ln.alive && ln.ndone < n_started;
        if (!__any(need)) break;
        if (need) {
          if (dt >= op.a) fail(ln, ST_HANG);
          else tick(x, ln);
        }
      }
      for (int32_t k = 0; k < op.b; ++k)
        if (ln.alive) tick(x, ln);
    }
  }

  // tokens still queued (the checkTokens residual, test_common.go:298-328)
  int32_t inflight = 0;
  {
    const uint32_t cap = 1u << lay.cap_log2;
    for (int32_t c = 0; c < p.n_ch; ++c) {
      const uint32_t chw = LW(lay.w_chw + c);
      const uint32_t cnt = (chw >> 8) & 0xffu, head = chw & 0xffu;
      for (uint32_t k = 0; k < cnt && k < cap; ++k) {
        const uint32_t e = LW(lay.w_fifo + ((uint32_t)c << lay.cap_log2) + ((head + k) & (cap - 1)));
        if (!(e & kMarkerBit)) inflight += (int32_t)(e & 0xffffu);
      }
      if (cnt > cap) {
        const uint32_t om = (1u << lay.ocap_log2) - 1;
        const uint32_t h = p.ovh[(int64_t)c * p.stride + ln.inst];
        for (uint32_t k = 0; k < cnt - cap; ++k) {
          const uint32_t e = p.ovf[(((int64_t)c << lay.ocap_log2) + ((h + k) & om)) * p.stride + ln.inst];
          if (!(e & kMarkerBit)) inflight += (int32_t)(e & 0xffffu);
        }
      }
    }
  }

  if (valid) {
    for (int32_t k = 0; k < lay.words; ++k) p.state[(int64_t)k * p.stride + ln.inst] = LW(k);
    int32_t* r = p.regs + ln.inst;
    r[R_TIME * p.stride] = ln.time;
    r[R_DRAW * p.stride] = ln.dptr;
    r[R_STATUS * p.stride] = ln.status;
    r[R_NDONE * p.stride] = ln.ndone;
    r[R_PEEK * p.stride] = (int32_t)ln.peek;
    r[R_POP_TOK * p.stride] = (int32_t)ln.pop_tok;
    r[R_POP_MK * p.stride] = (int32_t)ln.pop_mk;
    r[R_PUSH * p.stride] = (int32_t)ln.push;
    r[R_INFLIGHT_TOK * p.stride] = inflight;
  }
}

#undef LW

// Per-instance snapshot hash / conservation checks, summed over the batch.
__global__ __launch_bounds__(256) void cl_checksum_kernel(SumParams p) {
  const int64_t inst = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (inst >= p.n_inst) return;
  const int32_t* r = p.regs + inst;
  const int32_t st = r[R_STATUS * p.stride];
  unsigned long long v[10] = {1, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  if (st == ST_OK) v[1] = 1;
  else if (st == ST_FATAL_INSUFFICIENT || st == ST_FATAL_UNKNOWN_DEST) v[2] = 1;
  else v[3] = 1;
  if (st == ST_OK) {
    v[4] = (unsigned long long)(uint32_t)r[R_POP_TOK * p.stride] + (uint32_t)r[R_POP_MK * p.stride];
    const int32_t inflight = r[R_INFLIGHT_TOK * p.stride];
    v[9] = (unsigned long long)inflight;
    uint64_t hsum = 0, cut = 0;
    int64_t ncomplete = 0;
    for (int32_t sid = 0; sid < p.n_sids; ++sid) {
      if (p.snap_tick[(int64_t)sid * p.stride + inst] < 0) continue;
      ncomplete++;
      uint64_t h = 0x9E3779B97F4A7C15ULL ^ (uint64_t)sid;
      int64_t total = 0;
      for (int32_t n = 0; n < p.n_nodes; ++n) {
        const int32_t t = p.snap_tok[((int64_t)sid * p.n_nodes + n) * p.stride + inst];
        h = mix64(h ^ (uint64_t)(int64_t)t);
        total += t;
      }
      for (int32_t c = 0; c < p.n_ch; ++c) {
        const uint32_t rec = p.snap_rec[((int64_t)sid * p.n_ch + c) * p.stride + inst];
        const uint32_t b = rec & 0xffffu, e = rec >> 16;
        h = mix64(h ^ ((uint64_t)c << 32) ^ (uint64_t)(e - b));
        const int32_t* hv = p.hist_val + p.hist_off[c];
        for (uint32_t k = b; k < e; ++k) {
          h = mix64(h ^ (uint64_t)(int64_t)hv[k]);
          total += hv[k];
        }
      }
      hsum += h;
      const int64_t d = total - p.total_tokens;
      cut += (uint64_t)(d < 0 ? -d : d);
    }
    v[5] = hsum;
    v[6] = cut;
    v[8] = (unsigned long long)ncomplete;
    int64_t fin = inflight;
    for (int32_t n = 0; n < p.n_nodes; ++n)
      fin += (int32_t)p.state[(int64_t)(p.lay.w_tok + n) * p.stride + inst];
    const int64_t d = fin - p.total_tokens;
    v[7] = (unsigned long long)(d < 0 ? -d : d);
  }
  for (int k = 0; k < 10; ++k)
    if (v[k]) atomicAdd(&p.out[k], v[k]);
}

}  // namespace

int launch_exec(const ExecParams& p, const int32_t* topo, const Op* ops, const uint8_t* sched, void* stream) {
  const size_t lds = (size_t)p.lay.words * kWave * sizeof(uint32_t);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)cl_exec_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kMaxLdsBytes);
    if (e != hipSuccess) return (int)e;
  }
  const unsigned blocks = (unsigned)(p.stride / kWave);
  hipLaunchKernelGGL(cl_exec_kernel, dim3(blocks), dim3(kWave), lds, (hipStream_t)stream, p, topo, ops,
                     sched);
  return (int)hipGetLastError();
}

int launch_checksums(const SumParams& p, void* stream) {
  const unsigned blocks = (unsigned)((p.n_inst + 255) / 256);
  hipLaunchKernelGGL(cl_checksum_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, p);
  return (int)hipGetLastError();
}

}  // namespace clsnap
