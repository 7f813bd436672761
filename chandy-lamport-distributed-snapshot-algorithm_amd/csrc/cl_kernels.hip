// cl_kernels.hip -- gfx950 kernels of the Chandy-Lamport batch engine.
//
// cl_exec_kernel runs the event program (send / snapshot / tick / drain) for a batch of
// independent simulator instances.  Node-parallel layout: an instance of N nodes is a
// segment of N consecutive lanes of a 64-lane wave (lane = node rank), 64/N instances
// per wave, 4 independent waves per workgroup.  A node's mutable state lives in its
// lane: tokens and the STARTED mask in VGPRs (for degree bounds <= 4 also its out-links'
// head words, in-links' recording cursors and in-link match keys); its out-channel FIFOs,
// per-snapshot pending counters and trigger entries in the lane's private LDS column
// (word k at lds[k*64 + lane]: conflict-free for any per-lane index).  Lanes exchange
// three things per tick: the packet each sender picked (ds_bpermute reads of the sender's
// lane; the runtime-loop kernels of large degree bounds through a shared LDS region), the
// marker-broadcast draw counts and their exclusive prefix sums (shared LDS region, DPP
// scan).  HBM carries the delay schedule (1 B per draw, staged in LDS per wave) and the
// snapshot outputs.
//
// One tick (sim.go:71-95) in four wave-synchronous phases:
//   A pick     every sender scans its out-links in dest order and pops the first due head
//              (head-of-line; <= 1 delivery per sender).  Pushes made later in the same
//              tick can never be due in it, so picks from tick-start state are exact.
//   B receive  every receiver handles the picks addressed to it in ascending sender rank,
//              i.e. in the reference's delivery order: token -> tokens += n, cursor++;
//              marker -> CreateLocalSnapshot / close channel / completion (node.go:149-185).
//   C scan     first-receipt markers broadcast (node.go:97-109); the reference draws their
//              delays in sender order, so draw offsets are the exclusive prefix sum of
//              outdeg(receiver) over triggering senders (segmented wave scan).
//   D push     receivers push markers on their out-links with delays from those offsets.
// Reference map (paths relative to /root/reference/chandy_lamport): Tick sim.go:71-95,
// GetReceiveTime sim.go:100-102, StartSnapshot sim.go:105-123, NotifyCompletedSnapshot
// sim.go:126-131, CreateLocalSnapshot node.go:58-84, SendToNeighbors node.go:97-109,
// SendTokens node.go:112-131, HandleMarker node.go:149-171, HandleToken node.go:174-185,
// drain test_common.go:123-137.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include "cl_engine.h"

namespace clsnap {

#if CLSNAP_PROF
// Diagnostic build (make variant NAME=prof DEFS=-DCLSNAP_PROF=1): shader-clock cycles per
// program part, summed over waves.  [0] SEND ops, [1] SNAP ops, [2] tick phase A+B,
// [3] tick phase C/D, [4] drain/tick loop control, [5] prologue, [6] epilogue, [7] ticks.
__device__ unsigned long long g_prof[8];
#define PROF_T() ((unsigned long long)__builtin_readcyclecounter())
#else
#define PROF_T() 0ull
#endif

namespace {

// LDS pointers carry their address space explicitly: a generic pointer lets the compiler
// merge an LDS store with a global one into a FLAT store, and every FLAT op forces
// s_waitcnt vmcnt(0) lgkmcnt(0) -- a full memory drain inside the tick loop.
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef __attribute__((address_space(3))) uint8_t lds_u8;

// Uniform-per-lane context.  Output arrays are addressed with 32-bit element indices
// (the host keeps every array below 2^32 elements).
struct Ctx {
  const ExecParams& p;
  const Layout& lay;
  lds_u32* P;  // this lane's private column: word k at P[k * 64]
  lds_u32* X;  // this wave's LDS base (shared region at lay.x_*)
  const uint8_t* __restrict__ sched;  // delay schedule in HBM (row inst * sched_row)
  const lds_u8* lrow;                 // this instance's row staged in LDS (nullptr: read HBM)
  int32_t lane, seg_base, v, seg;
  uint32_t inst;      // instance index (0 for lanes without an instance)
  uint32_t stride;    // padded instance count
  int32_t indeg, outdeg, out_off;
  // snapshot outputs by 32-bit byte offsets from the (uniform) array bases: the stores use
  // the SGPR-base + 32-bit-VGPR-offset form, with no 64-bit address arithmetic per store
  uint32_t nod_plane8;  // bytes per sid plane of the node records / 256 (uniform; stride % 64 == 0)
  int32_t draws;       // delays per instance, clamped to int32 (draw indices are int32)
};

// Byte offset of snapshot plane `sid` (sid < 32): the plane is a multiple of 256 bytes (the
// instance stride is a multiple of 64), so sid * (plane / 256) fits the full-rate 24-bit
// multiplier (a generic 32-bit multiply is quarter rate) and the shift restores it.
__device__ __forceinline__ uint32_t plane_off(const Ctx& x, uint32_t sid, uint32_t plane8) {
  uint32_t m = __umul24(sid, plane8);
  asm volatile("" : "+v"(m));  // (else the compiler re-forms sid * plane: a quarter-rate multiply)
  return m << 8;
}
// This lane's byte offsets in snapshot plane 0, recomputed at each store (cheaper than
// keeping them live in VGPRs through the tick loop).
__device__ __forceinline__ uint32_t nod_lane(const Ctx& x) {
  return 4u * (x.inst * (uint32_t)x.p.n_nodes + (uint32_t)x.v) * (uint32_t)x.lay.rw;
}
// CLSNAP_ABL_NOSTORE (diagnostic timing builds only, results invalid): drop the snapshot
// output stores made during the tick loop, to price them.
#ifndef CLSNAP_ABL_NOSTORE
#define CLSNAP_ABL_NOSTORE 0
#endif
template <class T>
__device__ __forceinline__ void st_at(T* base, uint32_t byte_off, T val) {
  *reinterpret_cast<T*>(reinterpret_cast<char*>(base) + byte_off) = val;
}
template <class T>
__device__ __forceinline__ void st_snap(T* base, uint32_t byte_off, T val) {
  if constexpr (!CLSNAP_ABL_NOSTORE) st_at(base, byte_off, val);
}

// Append one Logger record (trace build only) for a traced instance.
template <bool TRACE>
__device__ __forceinline__ void temit(const Ctx& x, uint32_t kind, uint32_t other, int32_t epoch, uint32_t order,
                                      int32_t data, int32_t tokens) {
  if constexpr (TRACE) {
    const int64_t k = (int64_t)x.inst - x.p.trace_lo;
    if (k >= 0 && k < x.p.trace_n) {
      const uint32_t slot = atomicAdd(&x.p.trace_cnt[k], 1u);
      if (slot < (uint32_t)x.p.trace_cap) {
        TraceRec r;
        r.w0 = ((uint32_t)epoch & 0xffffu) | (kind << 16) | ((uint32_t)x.v << 19) | (other << 25);
        r.order = order;
        r.data = data;
        r.tokens = tokens;
        x.p.trace[k * x.p.trace_cap + slot] = r;
      }
    }
  }
}

struct Lane {
  int32_t tokens;
  uint32_t started;
  int32_t time, draw, status;
  uint32_t peek, push;
  uint32_t hw[2];   // (head words in registers, unrolled D <= 4) out-link k's head word: u16 k & 1 of word k >> 1
  uint32_t cur[2];  // (cursors in registers, unrolled D <= 4) in-link k's recording cursor: u16 k & 1 of word k >> 1
  bool alive;    // instance still running (uniform within the segment)
  int32_t flag;  // lane-local engine failure raised during an op/tick
#if CLSNAP_PROF
  unsigned long long prof[8];
#endif
};
#if CLSNAP_PROF
#define PROF_ADD(ln, k, t0) ((ln).prof[k] += PROF_T() - (t0))
#else
#define PROF_ADD(ln, k, t0) ((void)(t0))
#endif

// Small degree bounds keep loops unrolled and predicated with the in-link words in
// registers; larger ones use compact runtime loops over the node's own degree with the
// in-link words in the lane's LDS column (fewer VGPRs, one copy of the marker path).
// CLSNAP_UNROLL_MAX (cl_engine.h) is the largest D whose loops are unrolled; the unrolled
// phases A and B are predicated straight-line code (branchy forms measured slower, §9).
#ifndef CLSNAP_MAX_D
#define CLSNAP_MAX_D 128
#endif

constexpr bool unrolled(int D) { return D <= CLSNAP_UNROLL_MAX; }
template <int D>
using InLinks = uint32_t[unrolled(D) ? D : 1];
// The unrolled kernels hold each in-link as its match key: sender lane (bits 7..0) and the
// pick word's valid bit and out-link index at the sender (the bits of kKeyMask).  kNoKey
// (out-link 127 without the valid bit) matches no pick word.
constexpr uint32_t kKeyMask = 0x407f0000u;
constexpr uint32_t kNoKey = 0x007f0000u;
__device__ __forceinline__ uint32_t in_key(uint32_t w) {
  return (w & 0xffu) | ((w & 0x7f00u) << 8) | 0x40000000u;
}
// In-link recording cursors (delivered-token counts) of the unrolled kernels live in two
// packed registers instead of the link words' hi16 halves: phase B's per-in-link LDS read +
// write becomes one add (r03 A/B, §9).  The LDS halves are refreshed only for the state image.
// Out-link head words (8-bit ring head, 8-bit count) of the unrolled kernels live in two
// packed registers instead of the link words' lo16 halves: phase A's and the pushes' LDS
// reads + writes become register ops; the halves are refreshed for the epilogue (r04 A/B,
// gpurun_out/r04a: C3 2.380 -> 2.353 ms per step, C2 0.180 -> 0.176 ms).
constexpr bool hw_reg(int D) { return D <= 4 && CLSNAP_UNROLL_MAX >= D; }
constexpr bool cur_reg(int D) { return D <= 4 && unrolled(D); }

#define PW(k) (x.P[(uint32_t)(k) << 6])
#define XW(k) (x.X[(uint32_t)(k)])
// 16-bit half h of this lane's column word k: link word halves and trigger entries
#define PH(k, h) (reinterpret_cast<lds_u16*>(x.P + ((uint32_t)(k) << 6))[h])
// out-link ko's head word (lo16) and in-link ki's recording cursor (hi16) of link word k
#define CHW(ko) PH(lay.w_lnk + (ko), 0)
#define CUR(ki) PH(lay.w_lnk + (ki), 1)
// trigger entry k (16 bit: sender rank | snapshot id << 8)
#define TRIG(k) PH(lay.w_trig + ((uint32_t)(k) >> 1), (k) & 1)

// Out-link k's head word (k < D: a compile-time index in the unrolled kernels).
template <int D>
__device__ __forceinline__ uint32_t hw_get(const Ctx& x, const Lane& ln, int32_t k) {
  if constexpr (hw_reg(D)) return (ln.hw[k >> 1] >> ((k & 1) * 16)) & 0xffffu;
  const Layout& lay = x.lay;
  return CHW(k);
}
template <int D>
__device__ __forceinline__ void hw_set(const Ctx& x, Lane& ln, int32_t k, uint32_t v) {
  if constexpr (hw_reg(D)) {
    const uint32_t sh = (k & 1) * 16;
    ln.hw[k >> 1] = (ln.hw[k >> 1] & ~(0xffffu << sh)) | ((v & 0xffffu) << sh);
  } else {
    const Layout& lay = x.lay;
    CHW(k) = (uint16_t)v;
  }
}

// In-link k's recording cursor (k < D; a compile-time index in the unrolled kernels).
template <int D>
__device__ __forceinline__ uint32_t cur_get(const Ctx& x, const Lane& ln, int32_t k) {
  if constexpr (cur_reg(D)) return (ln.cur[k >> 1] >> ((k & 1) * 16)) & 0xffffu;
  const Layout& lay = x.lay;
  return CUR(k);
}
template <int D>
__device__ __forceinline__ void cur_add(const Ctx& x, Lane& ln, int32_t k, bool tok) {
  if constexpr (cur_reg(D)) {
    ln.cur[k >> 1] += tok ? (1u << ((k & 1) * 16)) : 0u;  // (<= 65,535 tokens per channel: no carry)
  } else {
    const Layout& lay = x.lay;
    const uint32_t c = CUR(k);
    CUR(k) = (uint16_t)(c + (tok ? 1u : 0u));
  }
}

// LDS atomic add (ds_add_rtn_u32); the wave's lanes are the only users of these words.
__device__ __forceinline__ uint32_t lds_add(lds_u32* a, uint32_t v) {
  return __atomic_fetch_add(a, v, __ATOMIC_RELAXED);
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Inclusive prefix sum over the 64 lanes with DPP (row shifts, then row broadcasts).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}

// Queue.Push (queue.go:18-20) on out-link ko; receiveTime = time + 1 + draw (sim.go:101).
// `k` is the index of the draw in this instance's delay stream.  STAGED: the wave's delay rows
// are staged in LDS.  A compile-time choice: with an HBM delay load anywhere on the path
// the compiler waits with s_waitcnt vmcnt(0) at the join, and on gfx950 vmcnt also counts
// the wave's outstanding global STORES (snapshot outputs) -- a full store drain per push.
// `pre`: the delay already read by the caller (PRE; a broadcast reads its delays together,
// one LDS wait instead of one per push).
template <int D, bool STAGED, bool PRE = false>
__device__ __forceinline__ void push(const Ctx& x, Lane& ln, int32_t ko, uint32_t payload, int32_t k,
                                     uint32_t pre = 0) {
  const Layout& lay = x.lay;
  if (k >= x.draws) { ln.flag = ST_DELAY_EXHAUSTED; return; }
  const uint32_t chw = hw_get<D>(x, ln, ko);
  const uint32_t cnt = chw >> 8;
  if (cnt >= (uint32_t)kMaxQueued) { ln.flag = ST_FIFO_OVERFLOW; return; }
  uint32_t delay;
  if constexpr (PRE) delay = pre;
  else if constexpr (STAGED) delay = x.lrow[k];
  else delay = x.sched[(size_t)x.inst * x.p.sched_row + k];
  const uint32_t e = payload | ((uint32_t)(ln.time + 1 + (int32_t)delay) << 16);
  const uint32_t cap = 1u << lay.cap_log2;
  if (__builtin_expect(cnt < cap, 1)) {
    PW(lay.w_fifo + ((uint32_t)ko << lay.cap_log2) + ((chw + cnt) & (cap - 1))) = e;
  } else {  // LDS ring full: younger packets of this channel spill to an HBM ring
    if (lay.ocap_log2 < 0 || cnt - cap >= (1u << lay.ocap_log2)) { ln.flag = ST_FIFO_OVERFLOW; return; }
    const uint32_t c = (uint32_t)(x.out_off + ko);
    const uint32_t om = (1u << lay.ocap_log2) - 1;
    uint32_t* hp = &x.p.ovh[c * x.stride + x.inst];
    // nothing spilled yet (cnt == cap): the ring restarts at slot 0, so its head needs no
    // reset per run -- spill rings are touched only by pushes that spill
    uint32_t h = 0;
    if (cnt == cap) *hp = 0u;
    else h = *hp;
    x.p.ovf[((c << lay.ocap_log2) + ((h + cnt - cap) & om)) * x.stride + x.inst] = e;
    if (x.p.spill_flag) x.p.spill_flag[x.inst] = 1;  // (the replay plan: this instance needs the rings)
  }
  hw_set<D>(x, ln, ko, chw + kCountOne);
  ln.push++;
}

// push() as straight-line code: the FIFO entry is written to its ring slot, or -- when the
// push does not land in the LDS ring (link past the out-degree, delay stream exhausted, ring
// full) -- to this lane's pick word in the shared region, which is dead after phase B (phase
// A writes it before any read).  SPILLOK: a full LDS ring spills to the HBM ring under a
// (rare) branch, as push().  The failure flags follow push(): delay exhaustion first, then
// overflow; a later link of the same broadcast still pushes.
template <int D, bool SPILLOK>
__device__ __forceinline__ void push_pred(const Ctx& x, Lane& ln, int32_t ko, bool on, uint32_t payload, int32_t k,
                                          uint32_t delay) {
  const Layout& lay = x.lay;
  const uint32_t cap = 1u << lay.cap_log2;
  const uint32_t chw = hw_get<D>(x, ln, ko);
  const uint32_t cnt = chw >> 8;
  const bool dly_ok = k < x.draws;
  const bool live = on && dly_ok;
  bool ok = live && cnt < cap;
  const uint32_t e = payload | ((uint32_t)(ln.time + 1 + (int32_t)delay) << 16);
  const uint32_t slot = lay.w_fifo + ((uint32_t)ko << lay.cap_log2) + ((chw + cnt) & (cap - 1));
  *(ok ? &PW(slot) : &XW(lay.x_pick + x.lane)) = e;
  if constexpr (SPILLOK) {
    if (__builtin_expect(live && cnt >= cap, 0)) {  // LDS ring full: the HBM spill ring
      if (lay.ocap_log2 >= 0 && cnt < (uint32_t)kMaxQueued && cnt - cap < (1u << lay.ocap_log2)) {
        const uint32_t c = (uint32_t)(x.out_off + ko);
        const uint32_t om = (1u << lay.ocap_log2) - 1;
        uint32_t* hp = &x.p.ovh[c * x.stride + x.inst];
        uint32_t h = 0;
        if (cnt == cap) *hp = 0u;
        else h = *hp;
        x.p.ovf[((c << lay.ocap_log2) + ((h + cnt - cap) & om)) * x.stride + x.inst] = e;
        if (x.p.spill_flag) x.p.spill_flag[x.inst] = 1;
        ok = true;
      }
    }
  }
  if constexpr (hw_reg(D)) ln.hw[ko >> 1] += ok ? kCountOne << ((ko & 1) * 16) : 0u;
  else hw_set<D>(x, ln, ko, ok ? chw + kCountOne : chw);
  ln.push += ok ? 1u : 0u;
  ln.flag = (on && !ok) ? (dly_ok ? (int32_t)ST_FIFO_OVERFLOW : (int32_t)ST_DELAY_EXHAUSTED) : ln.flag;
}

// CreateLocalSnapshot (node.go:58-84): record tokens and open every in-channel except
// the one the first marker arrived on (arrive = -1 at the initiator).  A channel's
// recording is the cursor interval [begin, end) over the tokens delivered on it.
template <int D>
__device__ __forceinline__ void create_local(const Ctx& x, Lane& ln, const InLinks<D>& it, int32_t sid,
                                             int32_t arrive) {
  const ExecParams& p = x.p;
  const Layout& lay = x.lay;
  const uint32_t rb = plane_off(x, (uint32_t)sid, x.nod_plane8) + nod_lane(x);
  if constexpr (unrolled(D)) {
    // the whole record in one vector store (RW words: a power of two, Layout::rw)
    constexpr int RW = D == 1 ? 2 : D <= 3 ? 4 : 8;
    uint32_t r[RW];
    r[0] = (uint32_t)ln.tokens;
#pragma unroll
    for (int32_t kj = 0; kj < RW - 1; ++kj) {
      const uint32_t cur = (kj < D && kj < x.indeg) ? cur_get<D>(x, ln, kj) : 0u;
      r[1 + kj] = kj == arrive ? (cur | (cur << 16)) : cur;
    }
    (void)it;
    if constexpr (RW == 2) {
      st_snap(reinterpret_cast<uint2*>(p.snap_nod), rb, make_uint2(r[0], r[1]));
    } else {
#pragma unroll
      for (int q = 0; q < RW; q += 4)
        st_snap(reinterpret_cast<uint4*>(p.snap_nod), rb + 4u * q, make_uint4(r[q], r[q + 1], r[q + 2], r[q + 3]));
    }
  } else {
    st_snap(p.snap_nod, rb, (uint32_t)ln.tokens);
    for (int32_t kj = 0; kj < x.indeg; ++kj) {
      const uint32_t cur = CUR(kj);
      st_snap(p.snap_nod, rb + 4u * (1 + kj), kj == arrive ? (cur | (cur << 16)) : cur);
    }
  }
}

// NotifyCompletedSnapshot (sim.go:126-131): the instance's snapshot completes when all N
// nodes have; one LDS counter per (instance, snapshot).
// (u8 counters, four per word: a count never exceeds N <= 64, so the add never carries)
__device__ __forceinline__ void node_complete(const Ctx& x, Lane& ln, int32_t sid) {
  const uint32_t sh = ((uint32_t)sid & 3u) * 8u;
  const uint32_t old = lds_add(&XW(x.lay.x_done + x.seg * x.lay.sp + (sid >> 2)), 1u << sh);
  if (((old >> sh) & 0xffu) + 1 == (uint32_t)x.p.n_nodes) {
    st_snap(x.p.snap_tick, 4u * (x.inst * (uint32_t)x.lay.s_cap + (uint32_t)sid), ln.time);
    lds_add(&XW(x.lay.x_ndone + x.seg), 1u);
  }
}

// Fold lane-local engine failures into the instance status (all lanes must call).
__device__ __forceinline__ void resolve_failures(const Ctx& x, Lane& ln) {
  const uint64_t any = __ballot(ln.flag != 0);
  if (__builtin_expect(any == 0, 1)) return;
  const int32_t N = x.p.n_nodes;
  const uint64_t seg_mask = N == 64 ? ~0ull : (((1ull << N) - 1) << x.seg_base);
  const uint64_t m = any & seg_mask;
  const int32_t src = m ? (int32_t)__builtin_ctzll(m) : x.lane;
  const int32_t code = __shfl(ln.flag, src);
  if (m && ln.alive) {
    ln.status = code;
    ln.alive = false;
  }
  ln.flag = 0;
}

template <int D>
__device__ __forceinline__ uint32_t in_word(const Ctx& x, const InLinks<D>& it, int32_t k) {
  if constexpr (unrolled(D)) return it[k];
  else return PW(x.lay.w_int + k);
}

// HandleMarker (node.go:149-171) for snapshot `sid` arriving on in-link ki from `src`.
template <int D, bool TRACE>
__device__ __forceinline__ void handle_marker(const Ctx& x, Lane& ln, const InLinks<D>& it, int32_t ki, uint32_t w,
                                              uint32_t src, int32_t sid, int32_t& ntrig) {
  const Layout& lay = x.lay;
  const uint32_t pi = lay.w_pend + (sid >> 2), sh = (sid & 3) * 8;
  const bool first = !((ln.started >> sid) & 1u);
  if (first) {  // first marker: record, then broadcast (phase D)
    ln.started |= 1u << sid;
    create_local<D>(x, ln, it, sid, ki);
    if constexpr (TRACE)  // SendToNeighbors' SentMsgRecords (node.go:100)
      for (int32_t j = 0; j < x.outdeg; ++j)
        temit<TRACE>(x, TK_SENT_MARKER, (uint32_t)x.p.ch_dest[x.out_off + j], ln.time, (src << 8) | (1u + j), sid,
                     ln.tokens);
    // the broadcast's draw slot (0 for a node without out-links: the slot stays 0 and the
    // trigger entry is not counted)
    XW(lay.x_tslot + x.seg_base + src) = (uint32_t)x.outdeg;
    TRIG(ntrig) = (uint16_t)(src | ((uint32_t)sid << 8));
    ntrig += x.outdeg ? 1 : 0;
  } else {  // later marker: stop recording this channel
    // hi16 of the cursor word: the channel's end.  The record's offset is pinned in one
    // VGPR (empty asm) so the in-link's constant folds into the store's immediate offset
    // instead of the compiler keeping a 64-bit base per in-link live through the tick loop.
    uint32_t rb = plane_off(x, (uint32_t)sid, x.nod_plane8) + nod_lane(x);
    asm volatile("" : "+v"(rb));
    st_snap(reinterpret_cast<uint16_t*>(x.p.snap_nod), rb + 4u * (1 + (uint32_t)ki) + 2u,
            (uint16_t)cur_get<D>(x, ln, ki));
  }
  // the pending count (u8 field sh of word pi) in one LDS atomic: a creation sets it to
  // indeg - 1 (the field is 0 before), a later marker takes one (the field is >= 1: a marker
  // is still expected), so neither carries into the neighbouring fields
  const uint32_t old = lds_add(&PW(pi), first ? (uint32_t)(x.indeg - 1) << sh : 0u - (1u << sh));
  const uint32_t pend = first ? (uint32_t)(x.indeg - 1) : ((old >> sh) & 0xffu) - 1;
  if (pend == 0) {
    node_complete(x, ln, sid);
    temit<TRACE>(x, TK_END, 0u, ln.time, (src << 8) | 255u, sid, ln.tokens);  // sim.go:127
  }
}

// Pop from a channel whose younger packets spilled: refill the freed LDS slot (the ring's
// new tail) with the oldest spilled packet.
__device__ __forceinline__ void refill(const Ctx& x, int32_t ko, uint32_t slot) {
  const Layout& lay = x.lay;
  const uint32_t c = (uint32_t)(x.out_off + ko);
  const uint32_t om = (1u << lay.ocap_log2) - 1;
  uint32_t* hp = &x.p.ovh[c * x.stride + x.inst];
  const uint32_t h = *hp;
  PW(slot) = x.p.ovf[((c << lay.ocap_log2) + h) * x.stride + x.inst];
  *hp = (h + 1) & om;
}

// Tick (sim.go:71-95) for every lane whose instance is `act` (uniform per segment).
// Must be reached by all lanes of the wave.  D bounds every node's in/out degree;
// it[] holds this node's in-link words.
// Returns true when no lane of the wave picked a packet: the tick ended after phase A (B, C
// and D would change nothing; phase A counted the peeks).
template <int D, bool STAGED, bool TRACE, bool NOSPILL = false>
__device__ __forceinline__ bool tick(const Ctx& x, Lane& ln, const InLinks<D>& it, bool act) {
  const Layout& lay = x.lay;
  const uint32_t cap = 1u << lay.cap_log2;
  const unsigned long long pt0 = PROF_T();
  ln.time += act ? 1 : 0;
  // ---- A: pick ------------------------------------------------------------
  uint32_t pick = 0, empty_scanned = 0;
  if constexpr (unrolled(D)) {
    bool scanning = act;
#pragma unroll
    for (int32_t ko = 0; ko < D; ++ko) {
      if (ko >= lay.od) break;  // uniform: the layout holds od out-links per lane
      const bool look = scanning && ko < x.outdeg;
      const uint32_t chw = hw_get<D>(x, ln, ko);
      const uint32_t cnt = chw >> 8;
      const uint32_t head = chw & (cap - 1);
      const uint32_t slot = lay.w_fifo + ((uint32_t)ko << lay.cap_log2) + head;
      const uint32_t e = PW(slot);
      empty_scanned |= (look && cnt == 0) ? (1u << ko) : 0u;
      const bool nonempty = look && cnt != 0;
      ln.peek += nonempty ? 1u : 0u;
      const uint32_t rt = (e >> 16) & 0x7fffu;
      const bool due = nonempty && (int32_t)rt <= ln.time;
      if (__builtin_expect(due && cnt > cap, 0)) refill(x, ko, slot);
      const uint32_t popped = ((cnt - 1) << 8) + ((head + 1) & (cap - 1));
      hw_set<D>(x, ln, ko, due ? popped : chw);
      pick = due ? ((e & (kMarkerBit | 0xffffu)) | kPickValid | ((uint32_t)ko << 16)) : pick;
      scanning = scanning && !due;
    }
  } else if (act) {
    bool done = false;
#pragma unroll
    for (int32_t ko = 0; ko < (unrolled(D) ? D : x.outdeg); ++ko) {
      if (ko >= x.outdeg) break;
      if (done) continue;
      const uint32_t chw = hw_get<D>(x, ln, ko);
      const uint32_t cnt = chw >> 8;
      if (!cnt) {
        empty_scanned |= 1u << ko;
        continue;
      }
      ln.peek++;
      const uint32_t head = chw & (cap - 1);
      const uint32_t slot = lay.w_fifo + ((uint32_t)ko << lay.cap_log2) + head;
      const uint32_t e = PW(slot);
      if ((int32_t)((e >> 16) & 0x7fffu) > ln.time) continue;
      if (__builtin_expect(cnt > cap, 0)) refill(x, ko, slot);
      hw_set<D>(x, ln, ko, ((cnt - 1) << 8) + ((head + 1) & (cap - 1)));
      pick = (e & (kMarkerBit | 0xffffu)) | kPickValid | ((uint32_t)ko << 16);
      done = true;
    }
  }
  // the unrolled receive phase reads pick words from the senders' lanes (ds_bpermute); the
  // runtime-loop one, under divergent control flow, from the shared region
  if constexpr (!unrolled(D)) {
    XW(lay.x_pick + x.lane) = pick;
    wave_sync();
  }
  if (!__ballot(pick != 0)) {
    PROF_ADD(ln, 2, pt0);
    return true;
  }
  // ---- B: receive, in ascending sender rank ---------------------------------
  int32_t ntrig = 0;
  if constexpr (unrolled(D)) {
    // the senders' pick words, read from their lanes (ds_bpermute: no LDS store, no wave
    // sync, no LDS alias that would pin the reads behind the marker path's stores), all
    // issued before the first is used: one LDS round trip per tick, not one per in-link
    uint32_t pks[D];
#pragma unroll
    for (int32_t ki = 0; ki < D; ++ki) {
      if (ki >= lay.id) break;
      pks[ki] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((x.seg_base + (it[ki] & 0xffu)) << 2), (int)pick);
    }
#pragma unroll
    for (int32_t ki = 0; ki < D; ++ki) {
      if (ki >= lay.id) break;  // uniform: the layout holds id in-links per lane
      const uint32_t w = it[ki];
      const uint32_t src = w & 0xffu;
      const uint32_t pk = pks[ki];
      // one masked compare against the in-link's key (in_key): a valid pick on the out-link
      // that feeds this in-link.  Lanes of inactive instances picked nothing (pick = 0), and
      // in-links past the node's in-degree hold kNoKey, so neither needs its own test.
      const bool m = ((pk ^ w) & kKeyMask) == 0u;
      const bool mk = m && (int32_t)pk < 0;
      const bool tok = m && (int32_t)pk >= 0;
      const uint32_t pay = pk & 0xffffu;
      if constexpr (TRACE)  // ReceivedMsgRecord (sim.go:86), the receiver's tokens before handling
        if (m) temit<TRACE>(x, mk ? TK_RECV_MARKER : TK_RECV_TOKEN, src, ln.time, src << 8, (int32_t)pay, ln.tokens);
      // HandleToken: tokens += data; the channel's recording cursor advances
      ln.tokens += tok ? (int32_t)pay : 0;
      cur_add<D>(x, ln, ki, tok);
      if (mk) handle_marker<D, TRACE>(x, ln, it, ki, w, src, (int32_t)pay, ntrig);
    }
  } else if (act) {
#pragma unroll
    for (int32_t ki = 0; ki < (unrolled(D) ? D : x.indeg); ++ki) {
      if (ki >= x.indeg) break;
      const uint32_t w = in_word<D>(x, it, ki);
      const uint32_t src = w & 0xffu;
      const uint32_t pk = XW(lay.x_pick + x.seg_base + src);
      if (!(pk & kPickValid) || ((pk >> 16) & 0x7fu) != ((w >> 8) & 0xffu)) continue;
      const uint32_t pay = pk & 0xffffu;
      temit<TRACE>(x, (pk & kMarkerBit) ? TK_RECV_MARKER : TK_RECV_TOKEN, src, ln.time, src << 8, (int32_t)pay,
                   ln.tokens);
      if (!(pk & kMarkerBit)) {  // HandleToken: tokens += data; the recording cursor advances
        ln.tokens += (int32_t)pay;
        cur_add<D>(x, ln, ki, true);
        continue;
      }
      handle_marker<D, TRACE>(x, ln, it, ki, w, src, (int32_t)pay, ntrig);
    }
  }
  // ---- C/D: broadcast draws in sender order, then push -------------------------
  const unsigned long long pt1 = PROF_T();
  PROF_ADD(ln, 2, pt0);
  if (__ballot(ntrig > 0)) {
    wave_sync();
    const uint32_t t = XW(lay.x_tslot + x.lane);
    XW(lay.x_tslot + x.lane) = 0;
    XW(lay.x_off + x.lane) = wave_incl_scan(t);
    wave_sync();
    const uint32_t base = x.seg_base > 0 ? XW(lay.x_off + x.seg_base - 1) : 0u;
    const uint32_t total = XW(lay.x_off + x.seg_base + x.p.n_nodes - 1) - base;
    for (int32_t kk = 0; kk < ntrig; ++kk) {
      const uint32_t tv = TRIG(kk);
      const uint32_t src = tv & 0xffu;
      const uint32_t sid = tv >> 8;
      // exclusive prefix of the triggering sender within the instance
      const int32_t k0 = ln.draw + (int32_t)(XW(lay.x_off + x.seg_base + src) - (uint32_t)x.outdeg - base);
      if constexpr (STAGED && hw_reg(D)) {
        // the broadcast's delays, read together (k0 + j may pass the schedule's end only in
        // an instance that push() then freezes; the staged rows stay inside the wave's LDS).
        // Only where the heads live in registers (hw_reg): push_pred writes channel j's head
        // back even for j >= outdeg (unchanged), which with LDS heads (D = 8..128) lands past
        // the lane's out-links -- for j >= priv - w_lnk past its column, in the next wave's
        // region (tests/test_gpu_parity.py::test_uneven_fan_out_runtime_loop_kernel)
        uint32_t dl[D];
#pragma unroll
        for (int32_t j = 0; j < D; ++j) dl[j] = x.lrow[k0 + j];
#pragma unroll
        for (int32_t j = 0; j < D; ++j) asm volatile("" : "+v"(dl[j]));
#pragma unroll
        for (int32_t j = 0; j < D; ++j) push_pred<D, !NOSPILL>(x, ln, j, j < x.outdeg, kMarkerBit | sid, k0 + j, dl[j]);
      } else {
#pragma unroll
        for (int32_t j = 0; j < D; ++j) {
          if (j >= x.outdeg) continue;
          push<D, STAGED>(x, ln, j, kMarkerBit | sid, k0 + j);
        }
      }
      // the reference scans this sender's links after the pushes when the trigger came from
      // a lower rank: every link that was empty at tick start gets peeked once more (once
      // per tick: the first such trigger clears the mask)
      if ((int32_t)src < x.v && empty_scanned) {
        ln.peek += (uint32_t)__builtin_popcount(empty_scanned);
        empty_scanned = 0;
      }
    }
    ln.draw += act ? (int32_t)total : 0;
  }
  resolve_failures(x, ln);
  PROF_ADD(ln, 3, pt1);
#if CLSNAP_PROF
  ln.prof[7] += 1;
#endif
  return false;
}

// SendTokens (node.go:112-131) of one send event: balance check, link lookup, push -- all
// at the sender.  Must be reached by all lanes of the wave.
template <int D, bool STAGED, bool TRACE>
__device__ __forceinline__ void send_one(const Ctx& x, Lane& ln, const Op& op, int32_t opi) {
  const bool me = ln.alive && x.v == op.a;
  const bool insufficient = me && ln.tokens < op.c;
  const bool fatal = ((__ballot(insufficient) >> (x.seg_base + op.a)) & 1ull) != 0;
  if constexpr (TRACE)  // SentMsgRecord (node.go:118): after the balance check, before the link check
    if (me && !insufficient)
      temit<TRACE>(x, TK_SENT_TOKEN, op.b >= 0 ? (uint32_t)x.p.ch_dest[x.out_off + op.b] : kTraceNoLink, ln.time,
                   0x80000000u | ((uint32_t)opi << 8), op.c, ln.tokens);
  if (me && !insufficient && op.b >= 0) {
    ln.tokens -= op.c;
#pragma unroll
    for (int32_t j = 0; j < D; ++j)  // static register indices for the out-link
      if (j == op.b) push<D, STAGED>(x, ln, j, (uint32_t)op.c, ln.draw);
  }
  if (ln.alive) {
    if (fatal) {
      ln.status = ST_FATAL_INSUFFICIENT;
      ln.alive = false;
    } else if (op.b < 0) {
      ln.status = ST_FATAL_UNKNOWN_DEST;
      ln.alive = false;
    } else {
      ln.draw += 1;
    }
  }
  resolve_failures(x, ln);
}

// A group of k send events with pairwise distinct senders (OP_SENDS): no event changes
// another's sender balance or channel, so when none of them fails every sender lane runs
// its own event at once, with draw index draw + its position in the group.  If any event
// of the wave would fail, the events run one by one (send_one), which freezes an instance
// exactly where the sequential program does.
template <int D, bool STAGED, bool TRACE>
__device__ __forceinline__ void send_group(const Ctx& x, Lane& ln, const Op* __restrict__ ev, int32_t k,
                                           int32_t opi0) {
  const Layout& lay = x.lay;
  int32_t pos = -1, oj = 0, on = 0;
  for (int32_t q = 0; q < k; ++q) {
    const Op s = ev[q];
    const bool me = x.v == s.a;
    pos = me ? q : pos;
    oj = me ? s.b : oj;
    on = me ? s.c : on;
  }
  const bool mine = ln.alive && pos >= 0;
  bool bad = false;
  if (mine) {
    if (ln.tokens < on || oj < 0 || ln.draw + pos >= x.draws) {
      bad = true;
    } else {  // the checks push() makes
      uint32_t chw = 0;
      if constexpr (hw_reg(D)) {
#pragma unroll
        for (int32_t j = 0; j < D; ++j) chw = j == oj ? hw_get<D>(x, ln, j) : chw;
      } else {
        chw = CHW(oj);
      }
      const uint32_t cnt = chw >> 8, cap = 1u << lay.cap_log2;
      bad = cnt >= (uint32_t)kMaxQueued || (cnt >= cap && (lay.ocap_log2 < 0 || cnt - cap >= (1u << lay.ocap_log2)));
    }
  }
  if (__builtin_expect(__ballot(bad) != 0, 0)) {
    for (int32_t q = 0; q < k; ++q) send_one<D, STAGED, TRACE>(x, ln, ev[q], opi0 + q);
    return;
  }
  if (mine) {
    temit<TRACE>(x, TK_SENT_TOKEN, (uint32_t)x.p.ch_dest[x.out_off + oj], ln.time,
                 0x80000000u | ((uint32_t)(opi0 + pos) << 8), on, ln.tokens);
    ln.tokens -= on;
#pragma unroll
    for (int32_t j = 0; j < D; ++j)
      if (j == oj) push<D, STAGED>(x, ln, j, (uint32_t)on, ln.draw + pos);
  }
  if (ln.alive) ln.draw += k;
}

// Occupancy target per degree bound (minimum waves per SIMD in the launch bound; 256-thread
// workgroups), the measured choices of §9: D = 3, 4 at 5 waves with HBM spill rings and 6
// without (6 and 7 with spill rings cost scratch spills); the others the compiler's choice.
constexpr int waves_for(int D, bool spill) { return (D == 3 || D == 4) ? (spill ? 5 : 6) : 1; }

// The whole event program for the instances of one wave (slots wave * ipw .. + ipw - 1 of
// the launch; n_slots slots in all).  Every lane of the wave must call it.
template <int D, bool STAGED, bool TRACE, int CAP, bool SPILL, bool MAPPED>
__device__ __forceinline__ void exec_wave(const ExecParams& p, const Layout& lay, uint32_t wave, uint32_t n_slots,
                                          const int32_t* imap, lds_u32* X, const uint32_t* __restrict__ topo,
                                          const Op* __restrict__ ops, const uint8_t* __restrict__ sched) {
  const int32_t N = p.n_nodes;
  const int32_t lane = threadIdx.x & (kWave - 1);
  const int32_t seg = lane / N;
  const int32_t v = lane - seg * N;
  // slot = position in the launch; inst = the instance it runs (imap: replays grouped by
  // length, spilling instances last, so a wave's segments finish together; cl_host.cpp)
  // (MAPPED: specialized kernels launch with a map, the others without; the generic CAP = 0
  // kernel checks at run time)
  const uint32_t slot = p.slot_base + wave * (uint32_t)lay.ipw + seg;
  const bool valid = seg < lay.ipw && slot < n_slots;
  const uint32_t inst = ((CAP > 0 || imap) && MAPPED && valid) ? (uint32_t)imap[slot] : slot;
  const uint32_t ii = valid ? inst : 0u;  // safe index for lanes without an instance
  const uint32_t* nb = topo + (size_t)(valid ? v : 0) * p.topo_w;
  const int32_t indeg = valid ? (int32_t)nb[0] : 0;
  const int32_t outdeg = valid ? (int32_t)nb[1] : 0;
  const uint32_t st = (uint32_t)p.stride;
  // Stage the wave's delay rows (ipw contiguous rows of sched_row bytes) in LDS when they fit.
  const lds_u8* lrow = STAGED ? (const lds_u8*)(X + lay.x_delay) + (size_t)seg * p.sched_row : nullptr;
  if constexpr (STAGED) {
    const uint32_t first = p.slot_base + wave * (uint32_t)lay.ipw;
    const uint32_t nrow = min((uint32_t)lay.ipw, n_slots - min(first, n_slots));
    const uint32_t rw4 = (uint32_t)(p.sched_row / 4);
    if (!MAPPED || (CAP == 0 && !imap)) {  // consecutive instances: one contiguous copy
      const uint32_t words = nrow * rw4;
      const uint32_t* src = reinterpret_cast<const uint32_t*>(sched + (size_t)first * p.sched_row);
      for (uint32_t k = lane; k < words; k += kWave) X[lay.x_delay + k] = src[k];
    } else {  // mapped slots: row by row
      for (uint32_t r = 0; r < nrow; ++r) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(sched + (size_t)imap[first + r] * p.sched_row);
        for (uint32_t k = lane; k < rw4; k += kWave) X[lay.x_delay + r * rw4 + k] = src[k];
      }
    }
  }
  const Ctx x{p, lay, X + lay.col + lane, X, sched, lrow, lane, seg * N, v, seg, ii, st,
              indeg, outdeg, valid ? (int32_t)nb[2] : 0,
              (4u * st * (uint32_t)N * (uint32_t)lay.rw) >> 8,
              (int32_t)(p.draws < 0x7fffffffLL ? p.draws : 0x7fffffffLL)};
  InLinks<D> it;
  if constexpr (unrolled(D)) {
#pragma unroll
    for (int32_t k = 0; k < D; ++k) it[k] = k < indeg ? in_key(nb[3 + k]) : kNoKey;
  } else {
    it[0] = 0;
  }

  Lane ln;
  ln.flag = 0;
#if CLSNAP_PROF
  for (int k = 0; k < 8; ++k) ln.prof[k] = 0;
  const unsigned long long pro0 = PROF_T();
#endif
  for (int32_t k = lane; k < lay.x_delay_begin; k += kWave) XW(k) = 0u;
  if (p.fresh) {
    // completion ticks start at -1 (no separate fill launch before every replay); the wait
    // orders these stores before any completion store of the same wave
    if (valid)
      for (int32_t sid = v; sid < lay.s_cap; sid += N)
        st_at(p.snap_tick, 4u * (x.inst * (uint32_t)lay.s_cap + (uint32_t)sid), (int32_t)-1);
    __builtin_amdgcn_s_waitcnt(0);
    for (int32_t k = 0; k < lay.priv; ++k) PW(k) = 0u;
    ln.tokens = valid ? (int32_t)topo[(size_t)N * p.topo_w + v] : 0;
    ln.started = 0;
    ln.time = ln.draw = ln.status = 0;
    ln.peek = ln.push = 0;
  } else {
    const uint32_t* S = p.state + ii;
    const uint32_t b = (uint32_t)v * (lay.priv + G_NUM);
    for (int32_t k = 0; k < lay.priv; ++k) PW(k) = valid ? S[(b + k) * st] : 0u;
    const uint32_t* R = S + (b + lay.priv) * st;
    ln.tokens = valid ? (int32_t)R[G_TOKENS * st] : 0;
    ln.started = valid ? R[G_STARTED * st] : 0;
    ln.time = valid ? (int32_t)R[G_TIME * st] : 0;
    ln.draw = valid ? (int32_t)R[G_DRAW * st] : 0;
    ln.status = valid ? (int32_t)R[G_STATUS * st] : 0;
    ln.peek = valid ? R[G_PEEK * st] : 0;
    ln.push = valid ? R[G_PUSH * st] : 0;
    wave_sync();
    if (valid && v == 0) {
      const uint32_t* Dn = S + (uint32_t)N * (lay.priv + G_NUM) * st;
      for (int32_t q = 0; q < lay.sp; ++q) {
        uint32_t w = 0;
        for (int32_t b = 0; b < 4; ++b) w |= (Dn[(4 * q + b) * st] & 0xffu) << (8 * b);
        XW(lay.x_done + seg * lay.sp + q) = w;
      }
      XW(lay.x_ndone + seg) = Dn[lay.s_cap * st];
    }
  }
  if constexpr (!unrolled(D))
    for (int32_t k = 0; k < indeg; ++k) PW(lay.w_int + k) = nb[3 + k];
  ln.cur[0] = ln.cur[1] = 0;
  ln.hw[0] = ln.hw[1] = 0;
  if constexpr (hw_reg(D)) {
#pragma unroll
    for (int32_t k = 0; k < D; ++k)
      if (k < lay.od) ln.hw[k >> 1] |= (uint32_t)CHW(k) << ((k & 1) * 16);
  }
  if constexpr (cur_reg(D)) {
#pragma unroll
    for (int32_t k = 0; k < D; ++k)
      if (k < indeg) ln.cur[k >> 1] |= (uint32_t)CUR(k) << ((k & 1) * 16);
  }
  wave_sync();
  ln.alive = valid && ln.status == ST_OK;
  int32_t n_started = p.n_started_before;
#if CLSNAP_PROF
  PROF_ADD(ln, 5, pro0);
#endif

  for (int32_t i = p.op_begin; i < p.op_end; ++i) {
    const Op op = ops[i];
    const unsigned long long ot0 = PROF_T();
    if (op.kind == OP_SEND) {
      send_one<D, STAGED, TRACE>(x, ln, op, i);
      PROF_ADD(ln, 0, ot0);
    } else if (op.kind == OP_SENDS) {
      send_group<D, STAGED, TRACE>(x, ln, ops + i + 1, op.a, i + 1);
      i += op.a;
      PROF_ADD(ln, 0, ot0);
    } else if (op.kind == OP_SNAP) {
      // sim.StartSnapshot -> node.StartSnapshot: the initiator records every in-channel
      if (ln.alive && v == op.a) {
        ln.started |= 1u << op.b;
        create_local<D>(x, ln, it, op.b, -1);
        if constexpr (TRACE) {  // StartSnapshotRecord (sim.go:109), then SendToNeighbors (node.go:100)
          const uint32_t o = 0x80000000u | ((uint32_t)i << 8);
          temit<TRACE>(x, TK_START, 0u, ln.time, o, op.b, ln.tokens);
          for (int32_t j = 0; j < outdeg; ++j)
            temit<TRACE>(x, TK_SENT_MARKER, (uint32_t)p.ch_dest[x.out_off + j], ln.time, o | (1u + j), op.b, ln.tokens);
        }
        const uint32_t pi = lay.w_pend + (op.b >> 2), sh = (op.b & 3) * 8;
        PW(pi) = (PW(pi) & ~(0xffu << sh)) | ((uint32_t)indeg << sh);
#pragma unroll
        for (int32_t j = 0; j < D; ++j)
          if (j < outdeg) push<D, STAGED>(x, ln, j, kMarkerBit | (uint32_t)op.b, ln.draw + j);
      }
      if (ln.alive) ln.draw += op.c;
      n_started++;
      resolve_failures(x, ln);
      PROF_ADD(ln, 1, ot0);
    } else if (op.kind == OP_TICK || op.kind == OP_DRAIN) {
      // TICK: op.a ticks.  DRAIN: tick until every started snapshot completed (at most
      // op.a ticks, else HANG), then op.b more (test_common.go:123-137).  Per instance.
      const bool drain = op.kind == OP_DRAIN;
      // A lane ticks while iter < until: op.a ticks, or (DRAIN) kNoUntil while it waits, and
      // op.b more from the iteration whose check finds its snapshots complete.  Every waiting
      // lane runs one tick per iteration, so the iteration count is its waiting ticks.  The
      // wait check runs only while some lane of the wave waits (uniform), so the tick loop's
      // control is one compare per iteration otherwise.
      constexpr int32_t kNoUntil = 0x7fffffff;
      int32_t until = drain ? kNoUntil : op.a;
      bool anyw = drain;
      for (int32_t iter = 0;; ++iter) {
        if (anyw) {
          const bool w = until == kNoUntil;
          if (w && (!ln.alive || (int32_t)XW(lay.x_ndone + seg) >= n_started)) {
            until = iter + op.b;
          } else if (w && iter >= op.a) {
            ln.status = ST_HANG;
            ln.alive = false;
            until = iter;
          }
          anyw = __ballot(until == kNoUntil) != 0;
        }
        const bool act = ln.alive && iter < until;
        if (!__ballot(act)) break;
        const bool idle = tick<D, STAGED, TRACE, (CAP > 0 && !SPILL)>(x, ln, it, act);
        if (idle && !anyw) {
          // nothing picked, and if nothing is queued anywhere in the wave either, every
          // remaining tick of this op is empty for every lane (no peek, draw or delivery: the
          // drain tail after the last delivery) -- add them at once
          uint32_t q = 0;
          if constexpr (hw_reg(D)) {
#pragma unroll
            for (int32_t k = 0; k < D; ++k)
              if (k < outdeg) q |= hw_get<D>(x, ln, k) >> 8;
          } else {
            for (int32_t k = 0; k < outdeg; ++k) q |= CHW(k) >> 8;
          }
          if (!__ballot(q != 0)) {
            if (ln.alive) ln.time += max(0, until - (iter + 1));
            break;
          }
        }
      }
#if CLSNAP_PROF
      PROF_ADD(ln, 4, ot0);
#endif
    }
  }
#if CLSNAP_PROF
  const unsigned long long epi0 = PROF_T();
#endif

  // ---- epilogue: tokens still queued, per-instance sums, outputs, state image ------
  if constexpr (hw_reg(D)) {  // the link words' head halves
#pragma unroll
    for (int32_t k = 0; k < D; ++k)
      if (k < lay.od) CHW(k) = (uint16_t)hw_get<D>(x, ln, k);
  }
  int32_t inflight = 0;
  {
    const uint32_t cap = 1u << lay.cap_log2;
    for (int32_t ko = 0; ko < outdeg; ++ko) {
      const uint32_t chw = CHW(ko);
      const uint32_t cnt = chw >> 8, head = chw & 0xffu;
      for (uint32_t k = 0; k < cnt && k < cap; ++k) {
        const uint32_t e = PW(lay.w_fifo + ((uint32_t)ko << lay.cap_log2) + ((head + k) & (cap - 1)));
        if (!(e & kMarkerBit)) inflight += (int32_t)(e & 0xffffu);
      }
      if (cnt > cap) {
        const uint32_t c = (uint32_t)(x.out_off + ko);
        const uint32_t om = (1u << lay.ocap_log2) - 1;
        const uint32_t h = p.ovh[c * st + ii];
        for (uint32_t k = 0; k < cnt - cap; ++k) {
          const uint32_t e = p.ovf[((c << lay.ocap_log2) + ((h + k) & om)) * st + ii];
          if (!(e & kMarkerBit)) inflight += (int32_t)(e & 0xffffu);
        }
      }
    }
  }
  // Queue.Pop counts (sim.go:85), derived instead of counted per tick: every pop delivers to
  // one receiver of the same instance in the same tick, so the instance's token pops are its
  // in-links' recording cursors (one per delivered token packet) and its marker pops are, per
  // started snapshot, indeg - pending (a creation's marker plus the later ones; an initiator
  // starts at indeg pending).
  uint32_t ptok = 0, pmk = 0;
  if constexpr (unrolled(D)) {
#pragma unroll
    for (int32_t k = 0; k < D; ++k)
      if (k < indeg) ptok += cur_get<D>(x, ln, k);
  } else {
    for (int32_t k = 0; k < indeg; ++k) ptok += CUR(k);
  }
  for (uint32_t m = ln.started; m; m &= m - 1u) {
    const uint32_t sid = (uint32_t)__builtin_ctz(m);
    pmk += (uint32_t)indeg - ((PW(lay.w_pend + (sid >> 2)) >> ((sid & 3u) * 8u)) & 0xffu);
  }
  if (valid) {
    lds_u32* acc = &XW(lay.x_acc + 5 * seg);
    lds_add(acc + 0, ln.peek);
    lds_add(acc + 1, ptok);
    lds_add(acc + 2, pmk);
    lds_add(acc + 3, ln.push);
    lds_add(acc + 4, (uint32_t)inflight);
  }
  wave_sync();
#if CLSNAP_PROF
  PROF_ADD(ln, 6, epi0);
  if (lane == 0) {
    ln.prof[4] -= ln.prof[2] + ln.prof[3];  // loop control only
    for (int k = 0; k < 8; ++k) atomicAdd(&g_prof[k], ln.prof[k]);
  }
#endif
  if (!valid) return;
  p.fin_tok[ii * (uint32_t)N + v] = ln.tokens;
  if (v == 0) {
    const lds_u32* acc = &XW(lay.x_acc + 5 * seg);
    int32_t* r = p.regs + (size_t)ii * R_NUM;  // one 36-byte row per instance
    r[R_TIME] = ln.time;
    r[R_DRAW] = ln.draw;
    r[R_STATUS] = ln.status;
    r[R_NDONE] = (int32_t)XW(lay.x_ndone + seg);
    r[R_PEEK] = (int32_t)acc[0];
    r[R_POP_TOK] = (int32_t)acc[1];
    r[R_POP_MK] = (int32_t)acc[2];
    r[R_PUSH] = (int32_t)acc[3];
    r[R_INFLIGHT_TOK] = (int32_t)acc[4];
  }
  if (!p.save_state) return;
  if constexpr (cur_reg(D)) {  // the link words' cursor halves, for the state image
#pragma unroll
    for (int32_t k = 0; k < D; ++k)
      if (k < indeg) CUR(k) = (uint16_t)cur_get<D>(x, ln, k);
  }
  uint32_t* S = p.state + ii;
  const uint32_t b = (uint32_t)v * (lay.priv + G_NUM);
  for (int32_t k = 0; k < lay.priv; ++k) S[(b + k) * st] = PW(k);
  uint32_t* R = S + (b + lay.priv) * st;
  R[G_TOKENS * st] = (uint32_t)ln.tokens;
  R[G_STARTED * st] = ln.started;
  R[G_TIME * st] = (uint32_t)ln.time;
  R[G_DRAW * st] = (uint32_t)ln.draw;
  R[G_STATUS * st] = (uint32_t)ln.status;
  R[G_PEEK * st] = ln.peek;
  R[G_POP_TOK * st] = ptok;  // (informational: a continuation derives them again)
  R[G_POP_MK * st] = pmk;
  R[G_PUSH * st] = ln.push;
  if (v == 0) {
    uint32_t* Dn = S + (uint32_t)N * (lay.priv + G_NUM) * st;
    for (int32_t s = 0; s < lay.s_cap; ++s) Dn[s * st] = (XW(lay.x_done + seg * lay.sp + (s >> 2)) >> ((s & 3) * 8)) & 0xffu;
    Dn[lay.s_cap * st] = XW(lay.x_ndone + seg);
  }
}

// CAP > 0: the layout's private column is ColumnC<D, CAP> (compile-time offsets: register
// pressure of the D = 3 kernel 95 VGPRs + 58 SGPR spills -> ~80 VGPRs, no spills); SPILL false
// compiles out the HBM spill rings.  CAP = 0 reads every offset from the runtime layout (any
// D, any ring size).  The grid covers slots [p.slot_base, p.n_inst).
template <int D, bool STAGED, bool TRACE, int CAP, bool SPILL, bool MAPPED>
__global__ __launch_bounds__(kWave * kWavesPerBlock, waves_for(D, SPILL)) void cl_exec_kernel(
    ExecParams p, const uint32_t* __restrict__ topo, const Op* __restrict__ ops, const uint8_t* __restrict__ sched) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  Layout lay_ = p.lay;
  if constexpr (CAP > 0) {
    using Col = ColumnC<D, CAP>;
    lay_.cap_log2 = CAP;
    lay_.od = lay_.id = D;
    lay_.w_fifo = Col::w_fifo;
    lay_.w_lnk = Col::w_lnk;
    lay_.w_int = Col::w_int;
    lay_.w_trig = Col::w_trig;
    lay_.w_pend = Col::w_pend;
    if constexpr (!SPILL) lay_.ocap_log2 = -1;
    lay_.x_pick = 0;
    lay_.x_tslot = kWave;
    lay_.x_off = 2 * kWave;
    lay_.x_done = 3 * kWave;
  }
  const Layout& lay = lay_;
  const int32_t wib = threadIdx.x / kWave;
  lds_u32* X = (lds_u32*)(lds + (size_t)wib * lay.wave_words);
  exec_wave<D, STAGED, TRACE, CAP, SPILL, MAPPED>(p, lay, blockIdx.x * (uint32_t)p.lay.wpb + wib, (uint32_t)p.n_inst,
                                                  MAPPED ? p.inst_map : nullptr, X, topo, ops, sched);
}

#undef PW
#undef XW

#if !defined(CLSNAP_PART) || CLSNAP_PART == 0
// Per-instance snapshot hash / conservation checks, summed over the batch.
__global__ __launch_bounds__(256) void cl_checksum_kernel(SumParams p) {
  const int64_t inst = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (inst >= p.n_inst) return;
  const int32_t* r = p.regs + inst * R_NUM;
  const int32_t st = r[R_STATUS];
  unsigned long long v[10] = {1, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  if (st == ST_OK) v[1] = 1;
  else if (st == ST_FATAL_INSUFFICIENT || st == ST_FATAL_UNKNOWN_DEST) v[2] = 1;
  else v[3] = 1;
  if (st == ST_OK) {
    v[4] = (unsigned long long)(uint32_t)r[R_POP_TOK] + (uint32_t)r[R_POP_MK];
    const int32_t inflight = r[R_INFLIGHT_TOK];
    v[9] = (unsigned long long)inflight;
    uint64_t hsum = 0, cut = 0;
    int64_t ncomplete = 0;
    for (int32_t sid = 0; sid < p.n_sids; ++sid) {
      if (p.snap_tick[inst * p.s_cap + sid] < 0) continue;
      ncomplete++;
      uint64_t h = 0x9E3779B97F4A7C15ULL ^ (uint64_t)sid;
      int64_t total = 0;
      const uint32_t* rb = p.snap_nod + ((int64_t)sid * p.stride + inst) * p.n_nodes * p.rw;
      for (int32_t n = 0; n < p.n_nodes; ++n) {
        const int32_t t = (int32_t)rb[(int64_t)n * p.rw];
        h = mix64(h ^ (uint64_t)(int64_t)t);
        total += t;
      }
      for (int32_t c = 0; c < p.n_ch; ++c) {
        const uint32_t rec = rb[p.ch_slot[c]];
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
    for (int32_t n = 0; n < p.n_nodes; ++n) fin += p.fin_tok[inst * p.n_nodes + n];
    const int64_t d = fin - p.total_tokens;
    v[7] = (unsigned long long)(d < 0 ? -d : d);
  }
  for (int k = 0; k < 10; ++k)
    if (v[k]) atomicAdd(&p.out[k], v[k]);
}

// Recorded copies over completed snapshots, all instances / OK instances (cl_get_counters).
__global__ __launch_bounds__(256) void cl_recorded_kernel(SumParams p) {
  const int64_t inst = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long rec = 0;
  bool ok = false;
  if (inst < p.n_inst) {
    ok = p.regs[inst * R_NUM + R_STATUS] == ST_OK;
    for (int32_t sid = 0; sid < p.n_sids; ++sid) {
      if (p.snap_tick[inst * p.s_cap + sid] < 0) continue;
      const uint32_t* rb = p.snap_nod + ((int64_t)sid * p.stride + inst) * p.n_nodes * p.rw;
      for (int32_t c = 0; c < p.n_ch; ++c) {
        const uint32_t r = rb[p.ch_slot[c]];
        rec += (r >> 16) - (r & 0xffffu);
      }
    }
  }
  unsigned long long a = rec, b = ok ? rec : 0;
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o);
    b += __shfl_xor(b, o);
  }
  if ((threadIdx.x & 63) == 0) {
    if (a) atomicAdd(&p.out[0], a);
    if (b) atomicAdd(&p.out[1], b);
  }
}

// ---- CollectSnapshot packed on the device (PackParams) ------------------------------
// count: one thread per instance -- tokenMap entries, completion flag, and the number of
// recorded messages over the channels (the cursor intervals' lengths).
__global__ __launch_bounds__(256) void cl_pack_count(PackParams p) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  const int64_t inst = p.lo + i;
  const bool done = p.snap_tick[inst * p.s_cap + p.sid] >= 0;
  const uint32_t* rb = p.snap_nod + ((int64_t)p.sid * p.stride + inst) * p.n_nodes * p.rw;
  long long cnt = 0;
  for (int32_t v = 0; v < p.n_nodes; ++v) p.tokens[i * p.n_nodes + v] = done ? (int32_t)rb[(int64_t)v * p.rw] : -1;
  if (done)
    for (int32_t c = 0; c < p.n_ch; ++c) {
      const uint32_t r = rb[p.ch_slot[c]];
      cnt += (long long)((r >> 16) - (r & 0xffffu));
    }
  p.complete[i] = done ? 1 : 0;
  p.count[i] = cnt;
}

// Exclusive scan of count[0, n) in place (count[n] = total): block-local scans of kScanItems
// entries (256 threads x 8, wave shuffles), a one-workgroup scan of the block sums, an add.
__device__ __forceinline__ long long block_scan_excl(long long x, long long* sh, long long* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  long long inc = x;
  for (int o = 1; o < 64; o <<= 1) {
    const long long y = __shfl_up(inc, o);
    if (lane >= o) inc += y;
  }
  if (lane == 63) sh[w] = inc;
  __syncthreads();
  long long pre = 0, tot = 0;
  for (int k = 0; k < (int)(blockDim.x >> 6); ++k) {
    if (k < w) pre += sh[k];
    tot += sh[k];
  }
  __syncthreads();
  *total = tot;
  return pre + inc - x;
}

__global__ __launch_bounds__(256) void cl_scan_blocks(long long* a, int64_t n, long long* bsum) {
  __shared__ long long sh[4];
  const int64_t base = (int64_t)blockIdx.x * kScanItems + threadIdx.x * 8;
  long long v[8], s = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    v[q] = base + q < n ? a[base + q] : 0;
    s += v[q];
  }
  long long tot;
  long long pre = block_scan_excl(s, sh, &tot);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    if (base + q < n) a[base + q] = pre;
    pre += v[q];
  }
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(256) void cl_scan_top(long long* bsum, int64_t nb, long long* total) {
  __shared__ long long sh[4];
  long long carry = 0;
  for (int64_t c0 = 0; c0 < nb; c0 += 256) {
    const int64_t k = c0 + threadIdx.x;
    const long long x = k < nb ? bsum[k] : 0;
    long long tot;
    const long long pre = block_scan_excl(x, sh, &tot);
    if (k < nb) bsum[k] = carry + pre;
    carry += tot;
  }
  if (threadIdx.x == 0) *total = carry;
}

__global__ __launch_bounds__(256) void cl_scan_add(long long* a, int64_t n, const long long* bsum) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] += bsum[i / kScanItems];
}

// fill: one thread per instance -- its channel offsets and its messages, channel by channel
// in delivery order (the token history interval [begin, end) of each recording cursor).
__global__ __launch_bounds__(256) void cl_pack_fill(PackParams p) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) p.offsets[p.n * p.n_ch] = p.count[p.n];
  if (i >= p.n) return;
  const int64_t inst = p.lo + i;
  const bool done = p.complete[i] != 0;
  const uint32_t* rb = p.snap_nod + ((int64_t)p.sid * p.stride + inst) * p.n_nodes * p.rw;
  long long m = p.count[i];
  long long* off = p.offsets + i * p.n_ch;
  for (int32_t c = 0; c < p.n_ch; ++c) {
    off[c] = m;
    if (!done) continue;
    const uint32_t r = rb[p.ch_slot[c]];
    const int32_t* hv = p.hist_val + p.hist_off[c];
    for (uint32_t k = r & 0xffffu; k < (r >> 16); ++k) p.msgs[m++] = hv[k];
  }
}

#endif

}  // namespace

// `stream`: launch there instead of L.stream, without the timing events unless `events`.
template <int D, bool STAGED, bool TRACE, int CAP = 0, bool SPILL = true, bool MAPPED = true>
int launch_exec_ds(const ExecParams& p, const uint32_t* topo, const Op* ops, const uint8_t* sched, const ExecLaunch& L,
                   void* stream = nullptr, bool events = false) {
  const int32_t wpb = p.lay.wpb;
  const size_t lds = (size_t)p.lay.wave_words * wpb * sizeof(uint32_t);
  auto* k = cl_exec_kernel<D, STAGED, TRACE, CAP, SPILL, MAPPED>;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, kMaxLdsBytes);
    if (e != hipSuccess) return (int)e;
  }
  const int64_t waves = (p.n_inst - p.slot_base + p.lay.ipw - 1) / p.lay.ipw;
  const unsigned blocks = (unsigned)((waves + wpb - 1) / wpb);
  if (blocks == 0) return 0;
  const bool ev = !stream || events;
  hipExtLaunchKernelGGL(k, dim3(blocks), dim3(kWave * wpb), lds, (hipStream_t)(stream ? stream : L.stream),
                        (hipEvent_t)(ev ? L.ev_start : nullptr), (hipEvent_t)(ev ? L.ev_stop : nullptr), 0u, p,
                        topo, ops, sched);
  return (int)hipGetLastError();
}

// A replay split by the plan of its first run (cl_host.cpp build_plan): the slot map puts the
// instances whose queues outgrew the LDS rings last; slots [0, split) run on the spill-free
// kernel (6 waves per SIMD for D = 3, 4), slots [split, n) on the spill-capable one,
// concurrently on a second stream (fork / join events).  The main dispatch records the start
// event and the stop event (a record after the join when joined); the spill-capable one its own pair.
template <int D, int CAP>
int launch_exec_split(const ExecParams& p, const uint32_t* topo, const Op* ops, const uint8_t* sched,
                      const ExecLaunch& L) {
  hipStream_t s = (hipStream_t)L.stream, s2 = (hipStream_t)L.stream2;
  hipError_t he;
  if (L.fork &&
      ((he = hipEventRecord((hipEvent_t)L.ev_fork, s)) || (he = hipStreamWaitEvent(s2, (hipEvent_t)L.ev_fork, 0))))
    return (int)he;
  ExecParams a = p, b = p;
  a.n_inst = p.split_slot;
  b.slot_base = (uint32_t)p.split_slot;
  ExecLaunch la = L;
  // the main dispatch records the start event and, unjoined, the stop event itself (a separate
  // record packet between back-to-back replays held the next dispatch ~8 us, gpurun_out/r05t)
  if (L.join) la.ev_stop = nullptr;
  // the spill-capable dispatch records start and stop events of its own (ev_start2 / ev_stop2):
  // unjoined, it may end after the main stream's stop, and the launch time is the longer half
  ExecLaunch lb = L;
  lb.ev_start = L.ev_start2;
  lb.ev_stop = L.ev_stop2;
  int e;
  // the spilling instances are the longest: their kernel is dispatched first so its
  // workgroups are resident from the start instead of queueing behind the main grid (the
  // tail of a small per-GPU batch)
  if ((e = launch_exec_ds<D, true, false, CAP, true, true>(b, topo, ops, sched, lb, s2, true))) return e;
  if ((e = launch_exec_ds<D, true, false, CAP, false, true>(a, topo, ops, sched, la))) return e;
  if (L.stop2_used && L.ev_stop2) *L.stop2_used = 1;
  if (!L.join) return 0;  // replays back to back: the main stream does not wait for stream2 (cl_host.cpp)
  if ((he = hipEventRecord((hipEvent_t)L.ev_join, s2)) || (he = hipStreamWaitEvent(s, (hipEvent_t)L.ev_join, 0)))
    return (int)he;
  if (L.ev_stop && (he = hipEventRecord((hipEvent_t)L.ev_stop, s))) return (int)he;
  return 0;
}

template <int D>
int launch_exec_d(const ExecParams& p, const uint32_t* topo, const Op* ops, const uint8_t* sched, const ExecLaunch& L) {
  // The trace build reads delays from HBM (one instantiation per D, debug runs only).
  if (p.trace_n > 0) return launch_exec_ds<D, false, true>(p, topo, ops, sched, L);
  if constexpr (unrolled(D)) {
    // staged delay rows and 2 / 4 / 8 LDS ring slots (every automatic choice): the kernel
    // specialized on the column layout, with or without HBM spill rings
    const bool ok = p.lay.od == D && p.lay.id == D;
    if (p.lay.x_delay > 0 && ok) {
      // spill rings in the layout: the spill-capable kernel, unless the replay plan knows the
      // program never spills (p.nospill) or splits the batch (p.split_slot)
      const bool rings = p.lay.ocap_log2 >= 0 && !p.nospill;
      const bool mp = p.inst_map != nullptr;
      const bool split = rings && mp && p.split_slot > 0 && p.split_slot < p.n_inst && L.stream2;
#define CLSNAP_SPEC(C)                                                                              \
  case C:                                                                                           \
    if (split) return launch_exec_split<D, C>(p, topo, ops, sched, L);                          \
    if (rings) return mp ? launch_exec_ds<D, true, false, C, true, true>(p, topo, ops, sched, L)   \
                         : launch_exec_ds<D, true, false, C, true, false>(p, topo, ops, sched, L); \
    return mp ? launch_exec_ds<D, true, false, C, false, true>(p, topo, ops, sched, L)          \
              : launch_exec_ds<D, true, false, C, false, false>(p, topo, ops, sched, L);
      switch (p.lay.cap_log2) {
        CLSNAP_SPEC(1)
        CLSNAP_SPEC(2)
        CLSNAP_SPEC(3)
        default: break;
      }
#undef CLSNAP_SPEC
    }
  }
  return p.lay.x_delay > 0 ? launch_exec_ds<D, true, false>(p, topo, ops, sched, L)
                           : launch_exec_ds<D, false, false>(p, topo, ops, sched, L);
}

// Build split (Makefile): this file is compiled once per degree set so the slow large-D
// instantiations build in parallel.  CLSNAP_PART 0 holds the dispatcher and the checksum
// kernel and references every launcher; CLSNAP_PART = D instantiates that D only.  Without
// CLSNAP_PART one translation unit holds every D up to CLSNAP_MAX_D (variant builds).
#if defined(CLSNAP_PART) && CLSNAP_PART > 0
template int launch_exec_d<CLSNAP_PART>(const ExecParams&, const uint32_t*, const Op*, const uint8_t*, const ExecLaunch&);
#else
#if defined(CLSNAP_PART)
extern template int launch_exec_d<1>(const ExecParams&, const uint32_t*, const Op*, const uint8_t*, const ExecLaunch&);
extern template int launch_exec_d<2>(const ExecParams&, const uint32_t*, const Op*, const uint8_t*, const ExecLaunch&);
extern template int launch_exec_d<3>(const ExecParams&, const uint32_t*, const Op*, const uint8_t*, const ExecLaunch&);
extern template int launch_exec_d<4>(const ExecParams&, const uint32_t*, const Op*, const uint8_t*, const ExecLaunch&);
extern template int launch_exec_d<8>(const ExecParams&, const uint32_t*, const Op*, const uint8_t*, const ExecLaunch&);
extern template int launch_exec_d<16>(const ExecParams&, const uint32_t*, const Op*, const uint8_t*, const ExecLaunch&);
extern template int launch_exec_d<32>(const ExecParams&, const uint32_t*, const Op*, const uint8_t*, const ExecLaunch&);
extern template int launch_exec_d<64>(const ExecParams&, const uint32_t*, const Op*, const uint8_t*, const ExecLaunch&);
extern template int launch_exec_d<128>(const ExecParams&, const uint32_t*, const Op*, const uint8_t*, const ExecLaunch&);
#endif
// The kernel is instantiated for degree bounds 1, 2, 3, 4, 8, ... CLSNAP_MAX_D.
int launch_exec(const ExecParams& p, const uint32_t* topo, const Op* ops, const uint8_t* sched, const ExecLaunch& L) {
  const int32_t d = p.lay.od > p.lay.id ? p.lay.od : p.lay.id;  // D must bound every in- and out-degree
  if (d <= 1) return launch_exec_d<1>(p, topo, ops, sched, L);
  if (d <= 2) return launch_exec_d<2>(p, topo, ops, sched, L);
  if (d <= 3) return launch_exec_d<3>(p, topo, ops, sched, L);  // 8nodes (BASELINE config 3)
  if (d <= 4) return launch_exec_d<4>(p, topo, ops, sched, L);
#if CLSNAP_MAX_D >= 8
  if (d <= 8) return launch_exec_d<8>(p, topo, ops, sched, L);
  if (d <= 16) return launch_exec_d<16>(p, topo, ops, sched, L);
  if (d <= 32) return launch_exec_d<32>(p, topo, ops, sched, L);
  if (d <= 64) return launch_exec_d<64>(p, topo, ops, sched, L);
  return launch_exec_d<128>(p, topo, ops, sched, L);
#else
  return (int)hipErrorNotSupported;
#endif
}

#if CLSNAP_PROF
extern "C" int cl_prof_read(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), sizeof(g_prof));
  if (e == hipSuccess && reset) {
    static const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof(z));
  }
  return (int)e;
}
#endif

int launch_checksums(const SumParams& p, void* stream) {
  const unsigned blocks = (unsigned)((p.n_inst + 255) / 256);
  hipLaunchKernelGGL(cl_checksum_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, p);
  return (int)hipGetLastError();
}

int launch_recorded(const SumParams& p, void* stream) {
  const unsigned blocks = (unsigned)((p.n_inst + 255) / 256);
  hipLaunchKernelGGL(cl_recorded_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, p);
  return (int)hipGetLastError();
}

int launch_pack_count(const PackParams& p, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (p.n > 0) {
    hipLaunchKernelGGL(cl_pack_count, dim3((unsigned)((p.n + 255) / 256)), dim3(256), 0, s, p);
    const int64_t nb = (p.n + kScanItems - 1) / kScanItems;
    hipLaunchKernelGGL(cl_scan_blocks, dim3((unsigned)nb), dim3(256), 0, s, p.count, p.n, p.bsum);
    hipLaunchKernelGGL(cl_scan_top, dim3(1), dim3(256), 0, s, p.bsum, nb, p.count + p.n);
    hipLaunchKernelGGL(cl_scan_add, dim3((unsigned)((p.n + 255) / 256)), dim3(256), 0, s, p.count, p.n,
                       (const long long*)p.bsum);
  } else {
    hipError_t e = hipMemsetAsync(p.count, 0, sizeof(long long), s);
    if (e != hipSuccess) return (int)e;
  }
  return (int)hipGetLastError();
}

int launch_pack_fill(const PackParams& p, void* stream) {
  const unsigned blocks = (unsigned)((p.n + 255) / 256);
  hipLaunchKernelGGL(cl_pack_fill, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, (hipStream_t)stream, p);
  return (int)hipGetLastError();
}

#endif  // CLSNAP_PART

}  // namespace clsnap
