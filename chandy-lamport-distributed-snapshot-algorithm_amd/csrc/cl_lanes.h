// cl_lanes.h -- the batch engine's instance-per-lane kernel, specialized on the topology.
//
// cl_exec_kernel (cl_kernels.hip) lays an instance of N nodes across N lanes: every wave
// instruction serves 64 / N instances, lanes exchange pick words and draw offsets, and most
// per-node work runs predicated on lanes with nothing to deliver (BASELINE config 3: ~2.4 of
// an instance's 8 lanes deliver in an average tick).  This kernel runs ONE instance per lane,
// 64 per wave.  Every instance of a batch has the same topology (the reference's .top file),
// so the topology is compiled into the kernel: cl_jit.cpp generates a topology type T (node
// count, degrees, CSR offsets, in-link senders) for the frozen topology and compiles this header
// with hipRTC for gfx950 at run time.  Every loop over node slots v < N and link slots is then
// unrolled with constant bounds and constant channel numbers: a node's state lives in
// registers of a fixed slot -- tokens, out-link head words, in-link recording cursors,
// per-snapshot pending nibbles -- and a sender's pick word reaches its receivers as a register
// read.  Only data-dependent addresses go through the lane's private LDS column (word k at
// lds[k * 64 + lane], conflict-free for any per-lane index): the FIFO rings (a head or tail
// slot differs per lane) and the instance's delay row.
//
// One tick (sim.go:71-95), exact in the reference's order:
//   A pick     every sender scans its out-links in dest order and pops the first due head;
//              picks from tick-start state are exact (a push made in tick t is due at >= t+1
//              and never changes a non-empty queue's head).
//   B receive  every receiver walks its in-links in ascending sender rank (the in-CSR order)
//              and handles the packet its sender picked for it: token -> tokens += n,
//              cursor++; marker -> CreateLocalSnapshot / close the channel (node.go:149-185).
//   C offsets  first-receipt markers broadcast (node.go:97-109) drawing their delays in
//              triggering-sender order: the exclusive prefix of the broadcasts' out-degrees
//              over senders.
//   D push     each receiver pushes its broadcasts on its out-links.
// Snapshot completion (sim.go:126-131) is one check per tick over the pending nibbles.
// Outputs, state image, spill rings and the replay plan are the node-parallel kernel's
// (cl_engine.h), so either kernel continues the other's launches.
// Reference map (paths relative to /root/reference/chandy_lamport): Tick sim.go:71-95,
// GetReceiveTime sim.go:100-102, StartSnapshot sim.go:105-123, NotifyCompletedSnapshot
// sim.go:126-131, CreateLocalSnapshot node.go:58-84, SendToNeighbors node.go:97-109,
// SendTokens node.go:112-131, HandleMarker node.go:149-171, HandleToken node.go:174-185,
// drain test_common.go:123-137.
//
// The topology type T provides (all constexpr):
//   N, D, SW             nodes, degree bound (every in- and out-degree <= D), pending words
//                        per node (8 snapshot ids each)
//   id(v), od(v)         in- and out-degree of node v
//   off(v)               first channel of node v (channels by (src rank, dest rank))
//   E, CAPL              channels, log2 of the LDS ring slots per channel
//   src(v, j), oix(v, j) in-link j of node v: sender rank and the link's out-index there
//   dst(v, k), ipos(v, k) out-link k of node v: receiver rank and the link's in-index there
#pragma once
#include "cl_engine.h"

namespace clsnap {
namespace lanes {

typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef const __attribute__((address_space(4))) ExecParams KPar;

// The kernel's parameters re-read from the kernarg segment (ExecParams is the first argument,
// at offset 0).  The empty asm makes every load through the pointer a fresh scalar load at its
// point of use instead of a value the compiler hoists out of the tick loop and keeps live.
__device__ __forceinline__ KPar* kpar() {
  auto* k = (const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(k));
  return (KPar*)k;
}

// Words per node snapshot record for degree bound D (rec_words of an unrolled layout).
constexpr int rec_w(int D) { return D == 1 ? 2 : D <= 3 ? 4 : 8; }

// Per-lane constants.
// LDS layout, per lane a private column:
//   FIFO rings, 16-bit entries: channel c's slot q is element (c << CAPL) + q, element i of
//   lane l at byte i * 128 + l * 2 (FW = E << CAPL >> 1 words of 256 bytes in all)
//   then 32-bit words, word w of lane l at byte w * 256 + l * 4:
//     FW            scratch word (stores that do not happen land here)
//     FW + 1 ..     the delay row, 8 nibbles per word (reads clamped to its last word: a
//                   window past the end only feeds pushes past `draws`, which fail anyway)
// A 16-bit FIFO entry: bits 7..0 receiveTime mod 256, bits 14..8 payload (token count or
// snapshot id, < 128), bit 15 marker.  receiveTime is recovered from its low byte because an
// entry is never more than draws + 4 ticks late when it is examined: while it is due but not
// delivered, either its queue's head is not yet due -- at most 4 ticks, as every packet behind
// a head was pushed no earlier and draws a delay of at most 4 -- or the sender delivers another
// packet that tick, and an instance delivers at most as many packets as it pushes (one draw
// each).  The host admits a program only with draws <= 240 (cl_jit.cpp lanes_fit), and an
// entry is due when (time - receiveTime) mod 256 < 251.
struct Ctx {
  uint32_t lb;      // this lane's byte offset in the 32-bit words: lane * 4
  uint32_t lb2;     // ... in the 16-bit FIFO elements: (lane & 31) * 4 + (lane >> 5) * 2
  uint32_t inst;    // instance of this lane (0 for lanes without one)
  uint32_t stride;
  uint32_t lrec;    // byte offset of this instance's node records in snapshot plane 0
  uint32_t plane8;  // bytes per snapshot plane / 256 (the stride is a multiple of 64)
  int32_t draws;    // delays per instance
  uint32_t dlast;   // column word of the delay row's last word
};

__device__ __forceinline__ lds_u32* lds_at(uint32_t byte) { return (lds_u32*)(size_t)byte; }
typedef __attribute__((address_space(3))) uint16_t lds_u16;
__device__ __forceinline__ lds_u16* lds16_at(uint32_t byte) { return (lds_u16*)(size_t)byte; }
// FIFO element i of this lane (cold paths: prologue, epilogue)
struct Ctx;
__device__ __forceinline__ uint32_t fifo_rd(const Ctx& x, uint32_t i);
__device__ __forceinline__ void fifo_wr(const Ctx& x, uint32_t i, uint32_t v);
__device__ __forceinline__ uint32_t fifo_rd(const Ctx& x, uint32_t i) { return *lds16_at(x.lb2 + (i << 7)); }
__device__ __forceinline__ void fifo_wr(const Ctx& x, uint32_t i, uint32_t v) { *lds16_at(x.lb2 + (i << 7)) = (uint16_t)v; }
__device__ __forceinline__ uint32_t col_rd(const Ctx& x, uint32_t w) { return *lds_at(x.lb + (w << 8)); }
__device__ __forceinline__ void col_wr(const Ctx& x, uint32_t w, uint32_t v) { *lds_at(x.lb + (w << 8)) = v; }

template <class T>
struct Lds {
  static constexpr uint32_t CAP = 1u << T::CAPL;
  static constexpr uint32_t CAPM7 = (CAP - 1u) << 7;  // a head word's ring-slot byte offset bits
  static constexpr uint32_t FW = ((uint32_t)T::E << T::CAPL) / 2;
  static constexpr uint32_t DUMMY = FW, DB = FW + 1;
  // words of a tick's delay window (reads past the row's end are clamped to its last word)
  static constexpr uint32_t WIN = (7 + T::E + 7) / 8 + 1;
};
// receiveTime <= time for a 16-bit entry (see the layout note): 1 or 0
__device__ __forceinline__ uint32_t due16(uint32_t e, int32_t time) {
  return (((((uint32_t)time - e) & 0xffu)) - 251u) >> 31;
}
// the node-parallel kernel's 32-bit entry (state image, HBM spill rings) and back
__device__ __forceinline__ uint32_t e16_to_32(uint32_t e, int32_t time) {
  const uint32_t rt = (uint32_t)time + 5u - (((uint32_t)time + 5u - e) & 0xffu);
  return ((e & 0x8000u) << 16) | ((e >> 8) & 0x7fu) | (rt << 16);
}
__device__ __forceinline__ uint32_t e32_to_16(uint32_t e) {
  return ((e >> 16) & 0xffu) | ((e & 0x7fu) << 8) | ((e >> 16) & 0x8000u);
}

// Delays k .. k + 7 of this instance as 4-bit nibbles (two column words, one ds_read2).
template <class T>
__device__ __forceinline__ uint32_t delays8(const Ctx& x, int32_t k) {
  const uint32_t w = Lds<T>::DB + ((uint32_t)min(k, x.draws) >> 3);
  const uint32_t lo = col_rd(x, min(w, x.dlast)), hi = col_rd(x, min(w + 1, x.dlast));
  return __builtin_amdgcn_alignbit(hi, lo, ((uint32_t)k & 7u) * 4u);
}

// Byte offset of snapshot plane `sid` on the full-rate 24-bit multiplier (cl_kernels.hip plane_off).
__device__ __forceinline__ uint32_t plane_off(const Ctx& x, uint32_t sid) {
  uint32_t m = __umul24(sid, x.plane8);
  asm volatile("" : "+v"(m));
  return m << 8;
}

template <class V>
__device__ __forceinline__ void st_at(V* base, uint32_t byte_off, V val) {
  *reinterpret_cast<V*>(reinterpret_cast<char*>(base) + byte_off) = val;
}

// The instruction scheduler may not move anything across this point: it keeps the unrolled
// node slots from being interleaved into one long region where every slot's lane masks are
// live at once (SGPR spills to VGPR lanes).
__device__ __forceinline__ void sched_fence() { __builtin_amdgcn_sched_barrier(0); }

// A value the optimizer cannot see through (op dispatch below).
template <class V>
__device__ __forceinline__ V opaque(V v) {
  asm volatile("" : "+v"(v));
  return v;
}

// Compile-time loop: f(IC<I>) for I in [B, E).
template <int I>
struct IC {
  static constexpr int value = I;
};
template <int B, int E, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (B < E) {
    f(IC<B>{});
    sfor<B + 1, E>(f);
  }
}

// State of one instance.
//   hw[v][k]  out-link k of node v: bits 6..0 queued packets (LDS ring + HBM spill; the host
//             admits a program only when no channel ever carries more than 127 packets), bits
//             7.. the ring head as a free-running counter (hw & CAPM7 = the head slot * 128)
//   cr[v][.]  in-link j's recording cursor (token packets delivered on the channel): u16 j & 1
//             of word j >> 1
//   pd[v][w]  per snapshot sid (w = sid >> 3) a nibble at 4 * (sid & 7): 0 not started,
//             pending + 1 after the node's local snapshot exists (1 = complete), 15 an initiator
//             without in-links (pending 0, but completion is only checked on a marker: never)
//   done[w]   bit 4 * (sid & 7) + 3 set once the instance's snapshot sid completed
template <class T>
struct State {
  int32_t tok[T::N];
  uint32_t hw[T::N][T::D];
  uint32_t cr[T::N][(T::D + 1) / 2];
  uint32_t pd[T::N][T::SW];
  uint32_t done[T::SW];
  int32_t time, draw, status, flag;
  uint32_t peek, push, ndone;
  bool alive;
};

template <class T>
__device__ __forceinline__ uint32_t cur_get(const State<T>& s, int v, int j) {
  return (s.cr[v][j >> 1] >> ((j & 1) * 16)) & 0xffffu;
}

// pending nibble word of a per-lane snapshot id (SW = 2: a select between the two words)
template <class T>
__device__ __forceinline__ uint32_t pd_get(const State<T>& s, int v, uint32_t sid) {
  if constexpr (T::SW == 1) return s.pd[v][0];
  else return (sid & 8u) ? s.pd[v][1] : s.pd[v][0];
}
template <class T>
__device__ __forceinline__ void pd_set(State<T>& s, int v, uint32_t sid, uint32_t w) {
  if constexpr (T::SW == 1) {
    s.pd[v][0] = w;
  } else {
    const bool hi = (sid & 8u) != 0;
    s.pd[v][1] = hi ? w : s.pd[v][1];
    s.pd[v][0] = hi ? s.pd[v][0] : w;
  }
}

// Queue.Push (queue.go:18-20) on channel ch (ring at column word ring) with receiveTime =
// time + 1 + delay (sim.go:101), draw index kd.  Straight-line: the entry goes to its ring slot
// or, when the push does not land in the ring, to the lane's scratch word.  SPILL: a full LDS
// ring spills to the HBM ring under a rare branch.  Failures follow the node-parallel kernel:
// delay exhaustion, then overflow; the node's last failing push sets nf.
template <class T, bool SPILL>
__device__ __forceinline__ void push(const Ctx& x, uint32_t& hw, uint32_t ch, bool on, uint32_t pl16, int32_t kd,
                                     uint32_t delay, int32_t time, uint32_t& npush, int32_t& nf) {
  using Ld = Lds<T>;
  const uint32_t cnt = hw & 0x7fu;
  const bool dly_ok = kd < x.draws;
  const bool live = on && dly_ok;
  bool ok = live && cnt < Ld::CAP;
  const uint32_t rt = (uint32_t)(time + 1 + (int32_t)delay);
  const uint32_t e = pl16 | (rt & 0xffu);
  // the ring slot (head + count) mod ring slots, its byte address, or the scratch word
  const uint32_t slot = (x.lb2 | ((hw + (hw << 7)) & Ld::CAPM7)) + (ch << (T::CAPL + 7));
  *lds16_at(ok ? slot : x.lb + (Ld::DUMMY << 8)) = (uint16_t)e;
  if constexpr (SPILL) {
    if (__builtin_expect(live && cnt >= Ld::CAP, 0)) {  // LDS ring full: the HBM spill ring
      KPar* p = kpar();
      const int32_t ocap = p->lay.ocap_log2;
      if (ocap >= 0 && cnt - Ld::CAP < (1u << ocap)) {
        const uint32_t om = (1u << ocap) - 1;
        uint32_t* hp = &p->ovh[ch * x.stride + x.inst];
        uint32_t h = 0;
        if (cnt == Ld::CAP) *hp = 0u;  // nothing spilled yet: the ring restarts at slot 0
        else h = *hp;
        p->ovf[((ch << ocap) + ((h + cnt - Ld::CAP) & om)) * x.stride + x.inst] =
            ((pl16 & 0x8000u) << 16) | ((pl16 >> 8) & 0x7fu) | (rt << 16);  // (the 32-bit entry)
        if (p->spill_flag) p->spill_flag[x.inst] = 1;
        ok = true;
      }
    }
  }
  hw += ok ? 1u : 0u;
  (void)npush;  // (pushes are derived at the epilogue: pops + packets still queued)
  nf = (on && !ok) ? (dly_ok ? (int32_t)ST_FIFO_OVERFLOW : (int32_t)ST_DELAY_EXHAUSTED) : nf;
}

// CreateLocalSnapshot (node.go:58-84) at node v: record tokens and open every in-channel except
// the one the first marker arrived on (arrive = -1 at the initiator): one vector store.
template <class T>
__device__ __forceinline__ void create_record(uint32_t* snod, const State<T>& s, int v, int arrive, uint32_t rb) {
  constexpr int RW = rec_w(T::D);
  uint32_t r[RW];
  r[0] = (uint32_t)s.tok[v];
#pragma unroll
  for (int j = 0; j < RW - 1; ++j) {
    const uint32_t c = (j < T::D && j < T::id(v)) ? cur_get(s, v, j < T::D ? j : 0) : 0u;
    r[1 + j] = j == arrive ? (c | (c << 16)) : c;
  }
  const uint32_t o = rb + (uint32_t)(v * RW * 4);
  if constexpr (RW == 2) {
    st_at(reinterpret_cast<uint2*>(snod), o, make_uint2(r[0], r[1]));
  } else {
#pragma unroll
    for (int q = 0; q < RW; q += 4)
      st_at(reinterpret_cast<uint4*>(snod), o + 4u * q, make_uint4(r[q], r[q + 1], r[q + 2], r[q + 3]));
  }
}

// Fold the lane's engine failure into its status (the instance freezes after the step).
template <class T>
__device__ __forceinline__ void resolve(State<T>& s) {
  if (s.flag != 0 && s.alive) {
    s.status = s.flag;
    s.alive = false;
  }
  s.flag = 0;
}

// Tick (sim.go:71-95) for a lane whose instance is `act`.  Every lane of the wave calls it.
// Returns true when no lane of the wave picked a packet (the tick ended after phase A).
template <class T, bool SPILL>
__device__ __forceinline__ bool tick(const Ctx& x, State<T>& s, bool act) {
  constexpr int N = T::N, D = T::D;
  s.time += act ? 1 : 0;
  // ---- A: pick ------------------------------------------------------------------------
  // every head first (independent LDS reads), then the scan
  uint32_t e[N][D];
#pragma unroll
  for (int v = 0; v < N; ++v)
#pragma unroll
    for (int k = 0; k < D; ++k)
      if (k < T::od(v))
        e[v][k] = lds16_at(x.lb2 | (s.hw[v][k] & Lds<T>::CAPM7))[(T::off(v) + k) << (T::CAPL + 6)];
  uint32_t pk[N];  // sender v's pick: (out-index + 1) << 16 | the 16-bit entry (0: nothing)
  uint32_t es[N];  // sender v's out-links that were empty when it scanned them
  // 0/1 integers in VGPRs, kept opaque: as compare masks the compiler would keep every
  // channel's masks live in SGPR pairs across the phase (and spill them to VGPR lanes)
#pragma unroll
  for (int v = 0; v < N; ++v) {
    pk[v] = 0;
    es[v] = 0;
    uint32_t sc = opaque(act ? 1u : 0u);  // still scanning
#pragma unroll
    for (int k = 0; k < D; ++k) {
      if (k >= T::od(v)) continue;
      const uint32_t w = s.hw[v][k];
      const uint32_t ne = opaque(min(w & 0x7fu, 1u));      // queue non-empty
      const uint32_t le = opaque(due16(e[v][k], s.time));  // receiveTime <= time
      const uint32_t lk = sc & ne;  // Peek (sim.go:83)
      s.peek += lk;
      es[v] |= (sc - lk) << k;
      const uint32_t due = opaque(lk & le);
      if constexpr (SPILL) {
        if (__builtin_expect(due && (w & 0x7fu) > Lds<T>::CAP, 0)) {  // refill the freed slot from the spill ring
          KPar* p = kpar();
          const uint32_t c = T::off(v) + k;
          const int32_t ocap = p->lay.ocap_log2;
          uint32_t* hp = &p->ovh[c * x.stride + x.inst];
          const uint32_t h = *hp;
          lds16_at(x.lb2 | (w & Lds<T>::CAPM7))[c << (T::CAPL + 6)] =
              (uint16_t)e32_to_16(p->ovf[((c << ocap) + h) * x.stride + x.inst]);
          *hp = (h + 1) & ((1u << ocap) - 1);
        }
      }
      s.hw[v][k] = w + due * 0x7fu;  // Pop: head + 1, count - 1
      const uint32_t val = e[v][k] | ((uint32_t)(k + 1) << 16);
      pk[v] = (val & (0u - due)) | (pk[v] & (due - 1u));
      sc -= due;
    }
    sched_fence();
  }
  // nothing due anywhere in the wave (15 % of C3's wave-ticks, mostly drain tails): the tick
  // ends here -- phase A already counted its peeks, and B, the completion check and C/D
  // would change nothing
  {
    uint32_t any = 0;
#pragma unroll
    for (int v = 0; v < N; ++v) any |= pk[v];
    if (!__ballot(any != 0)) return true;
  }
  // ---- B: receive, in-links in ascending sender rank ----------------------------------------
  // Straight-line and predicated: every register update happens on every lane (selects), only
  // the two snapshot-record stores sit in (divergent) branches -- register writes inside a
  // divergent branch make the compiler copy whole register tuples at the join.
  uint32_t tq[N];  // receiver v's first-marker triggers this tick: byte j = 0x80 | sid
  bool mkev = false;
  uint32_t* const snod = kpar()->snap_nod;
#pragma unroll
  for (int v = 0; v < N; ++v) {
    tq[v] = 0;
#pragma unroll
    for (int j = 0; j < D; ++j) {
      if (j >= T::id(v)) continue;
      const int sj = T::src(v, j);
      const uint32_t pkj = pk[sj];
      const bool m = (pkj >> 16) == (uint32_t)(T::oix(v, j) + 1);
      const bool mk = m && (pkj & 0x8000u);
      const bool tk = m && !(pkj & 0x8000u);
      // HandleToken (node.go:174-185): tokens += data, the channel's recording cursor advances
      s.tok[v] += tk ? (int32_t)((pkj >> 8) & 0x7fu) : 0;
      s.cr[v][j >> 1] += tk ? (1u << ((j & 1) * 16)) : 0u;
      // HandleMarker (node.go:149-171): the first marker of a snapshot creates the local
      // snapshot (pending = indeg - 1, nibble indeg) and triggers the broadcast; a later one
      // closes the channel (pending - 1)
      mkev = mkev || mk;
      const uint32_t sid = (pkj >> 8) & 31u;
      const uint32_t sh = (sid & 7u) * 4u;
      uint32_t pw = pd_get(s, v, sid);
      const bool nz = ((pw >> sh) & 15u) != 0;
      const bool first = mk && !nz, later = mk && nz;
      pw += first ? ((uint32_t)T::id(v) << sh) : later ? (0u - (1u << sh)) : 0u;
      pd_set(s, v, sid, pw);
      if (T::od(v) > 0) {
        tq[v] |= first ? (0x80u | sid) << (8 * j) : 0u;
        // the reference scans this sender's links after the pushes when the trigger came
        // from a lower rank: each link that was empty when it scanned it is peeked again
        if (T::src(v, j) < v) {
          s.peek += first ? (uint32_t)__builtin_popcount(es[v]) : 0u;
          es[v] = first ? 0u : es[v];
        }
      }
      const uint32_t rb = plane_off(x, sid) + x.lrec;
      if (first) create_record<T>(snod, s, v, j, rb);
      if (later)  // the channel's end cursor
        st_at(reinterpret_cast<uint16_t*>(snod), rb + (uint32_t)(v * rec_w(D) * 4 + 4 * (1 + j) + 2),
              (uint16_t)cur_get(s, v, j));
    }
    sched_fence();
  }
  // ---- NotifyCompletedSnapshot (sim.go:126-131): every node's nibble is 1 ---------------
  if (__ballot(mkev)) {
#pragma unroll
    for (int w = 0; w < T::SW; ++w) {
      uint32_t all = 0x88888888u;
#pragma unroll
      for (int v = 0; v < N; ++v) {
        const uint32_t y = s.pd[v][w] ^ 0x11111111u;  // nibble == 1 -> 0
        all &= ~(((y & 0x77777777u) + 0x77777777u) | y);
      }
      uint32_t fresh = all & 0x88888888u & ~s.done[w];
      if (fresh) {
        KPar* p = kpar();
        int32_t* tick_row = p->snap_tick + x.inst * (uint32_t)p->lay.s_cap;
        while (fresh) {
          const uint32_t b = (uint32_t)__builtin_ctz(fresh);
          tick_row[(uint32_t)w * 8u + (b >> 2)] = s.time;
          s.ndone += 1;
          s.done[w] |= 1u << b;
          fresh &= fresh - 1u;
        }
      }
    }
  }
  // ---- C/D: broadcast draws in triggering-sender order, then push ------------------------
  bool trig = false;
#pragma unroll
  for (int v = 0; v < N; ++v) trig = trig || tq[v] != 0;
  if (__ballot(trig)) {
    // C: sender s's delivery went out on one of its out-links; if it triggered a broadcast at
    // that link's receiver, the broadcast draws od(receiver) delays.  Exclusive offsets in
    // sender order (sim.go:101 draws in Tick's sender order).
    uint32_t off[N];
    uint32_t acc = 0;
#pragma unroll
    for (int sv = 0; sv < N; ++sv) {
      off[sv] = acc;
#pragma unroll
      for (int k = 0; k < D; ++k) {
        if (k >= T::od(sv)) continue;
        const int r = T::dst(sv, k), q = T::ipos(sv, k);
        acc += ((tq[r] >> (8 * q + 7)) & 1u) * (uint32_t)T::od(r);
      }
    }
    // the tick's delays in one LDS round trip: draws [draw, draw + acc) lie in the WN words
    // from draw / 8 (acc <= E: each channel carries at most one broadcast push per tick)
    constexpr int WN = (int)Lds<T>::WIN;
    uint32_t dw[WN];
    {
      const uint32_t w0 = Lds<T>::DB + ((uint32_t)min(s.draw, x.draws) >> 3);
#pragma unroll
      for (int q = 0; q < WN; ++q) dw[q] = col_rd(x, min(w0 + q, x.dlast));
    }
#pragma unroll
    for (int v = 0; v < N; ++v) {
      if (T::od(v) == 0) continue;
      int32_t nf = 0;
      while (__ballot(tq[v] != 0)) {  // usually once: one trigger per receiver and tick
        const uint32_t q = tq[v];
        const bool on = q != 0;
        const uint32_t lb = q ? (uint32_t)__builtin_ctz(q) & 24u : 0u;  // 8 * in-link
        const uint32_t sid = (q >> lb) & 31u;
        tq[v] = q & ~(0xffu << lb);
        uint32_t o = off[T::src(v, 0)];
#pragma unroll
        for (int j = 1; j < D; ++j)
          if (j < T::id(v)) o = lb == (uint32_t)(8 * j) ? off[T::src(v, j)] : o;
        const int32_t k0 = s.draw + (int32_t)o;
        // delays k0 .. k0 + 7: nibble i = (draw & 7) + o of the window
        const uint32_t i = ((uint32_t)s.draw & 7u) + (on ? o : 0u);
        uint32_t lo = dw[0], hi = dw[1];
#pragma unroll
        for (int q = 1; q + 1 < WN; ++q) {
          lo = (i >> 3) == (uint32_t)q ? dw[q] : lo;
          hi = (i >> 3) == (uint32_t)q ? dw[q + 1] : hi;
        }
        const uint32_t dl = __builtin_amdgcn_alignbit(hi, lo, (i & 7u) * 4u);
#pragma unroll
        for (int k = 0; k < D; ++k) {
          if (k >= T::od(v)) continue;
          push<T, SPILL>(x, s.hw[v][k], T::off(v) + k, on, 0x8000u | (sid << 8), k0 + k, (dl >> (4 * k)) & 15u,
                         s.time, s.push, nf);
        }
      }
      s.flag = s.flag ? s.flag : nf;  // the lowest-ranked failing node sets the status
    }
    s.draw += (int32_t)acc;
  }
  resolve(s);
  return false;
}

// Host ops name their node (and link) by uniform indices.  They are straight-line: the node's
// registers are picked with selects on the uniform index, and written back the same way, so no
// branch per node slot leaves the compiler a merge of every node's registers to resolve (those
// merges cost more registers than the tick itself).  The empty asm keeps the optimizer from
// folding a select chain over an array into one dynamically indexed access, which would move
// the instance state out of registers into scratch memory.
template <int N, class V>
__device__ __forceinline__ V pick_slot(const V (&a)[N], int32_t i) {
  V r = opaque(a[0]);
#pragma unroll
  for (int v = 1; v < N; ++v) r = v == i ? opaque(a[v]) : r;
  return r;
}
template <class T>
__device__ __forceinline__ uint32_t pick_hw(const State<T>& s, int32_t a, int32_t k) {
  uint32_t r = 0;
#pragma unroll
  for (int v = 0; v < T::N; ++v)
#pragma unroll
    for (int j = 0; j < T::D; ++j)
      if (j < T::od(v)) r = (v == a && j == k) ? opaque(s.hw[v][j]) : r;
  return r;
}

// SendTokens (node.go:112-131) of one send event: balance check, link lookup, push.
template <class T, bool SPILL>
__device__ __forceinline__ void send_one(const Ctx& x, State<T>& s, const Op& op) {
  const int32_t a = op.a, b = op.b;
  const int32_t tk = pick_slot<T::N>(s.tok, a);
  const bool insufficient = s.alive && tk < op.c;
  const bool go = s.alive && !insufficient && b >= 0;
  uint32_t hw = pick_hw(s, a, b);
  const uint32_t h0 = hw;
  int32_t nf = 0;
  const uint32_t ch = (uint32_t)(b >= 0 ? b : 0) + [&] {
    uint32_t o = 0;
#pragma unroll
    for (int v = 0; v < T::N; ++v) o = v == a ? T::off(v) : o;
    return o;
  }();
  push<T, SPILL>(x, hw, ch, go, (uint32_t)op.c << 8, s.draw, delays8<T>(x, s.draw) & 15u, s.time, s.push, nf);
  const uint32_t inc = hw - h0;  // 1 where the push landed
#pragma unroll
  for (int v = 0; v < T::N; ++v) {
    s.tok[v] -= (v == a && go) ? op.c : 0;
#pragma unroll
    for (int j = 0; j < T::D; ++j)
      if (j < T::od(v)) s.hw[v][j] += (v == a && j == b) ? inc : 0u;
  }
  s.flag = nf;
  if (s.alive) {
    if (insufficient) {
      s.status = ST_FATAL_INSUFFICIENT;
      s.alive = false;
    } else if (b < 0) {
      s.status = ST_FATAL_UNKNOWN_DEST;
      s.alive = false;
    } else {
      s.draw += 1;
    }
  }
  resolve(s);
}

// sim.StartSnapshot -> node.StartSnapshot (sim.go:105-123, node.go:198-212): the initiator
// records every in-channel and broadcasts.
template <class T, bool SPILL>
__device__ __forceinline__ void start_snapshot(const Ctx& x, State<T>& s, const Op& op) {
  constexpr int RW = rec_w(T::D);
  const int32_t a = op.a;
  const uint32_t sid = (uint32_t)op.b;
  const bool on = s.alive;
  int32_t id = 0, od = 0;
  uint32_t off = 0;
#pragma unroll
  for (int v = 0; v < T::N; ++v) {
    id = v == a ? T::id(v) : id;
    od = v == a ? T::od(v) : od;
    off = v == a ? T::off(v) : off;
  }
  // the pending nibble: pending = indeg (15: an initiator without in-links never completes)
  const uint32_t nib = (id == 0 ? 15u : (uint32_t)id + 1u) << ((sid & 7u) * 4u);
#pragma unroll
  for (int v = 0; v < T::N; ++v)
#pragma unroll
    for (int w = 0; w < T::SW; ++w) s.pd[v][w] |= (on && v == a && (uint32_t)w == (sid >> 3)) ? nib : 0u;
  // CreateLocalSnapshot (node.go:58-84) with every in-channel recording: one vector store
  uint32_t r[RW];
  r[0] = (uint32_t)pick_slot<T::N>(s.tok, a);
#pragma unroll
  for (int j = 0; j < RW - 1; ++j) {
    uint32_t c = 0;
    if (j < T::D) {
#pragma unroll
      for (int v = 0; v < T::N; ++v)
        if (j < T::id(v)) c = v == a ? opaque(cur_get(s, v, j)) : c;
    }
    r[1 + j] = c;
  }
  if (on) {
    const uint32_t o = plane_off(x, sid) + x.lrec + (uint32_t)a * (RW * 4u);
    uint32_t* snod = kpar()->snap_nod;
    if constexpr (RW == 2) {
      st_at(reinterpret_cast<uint2*>(snod), o, make_uint2(r[0], r[1]));
    } else {
#pragma unroll
      for (int q = 0; q < RW; q += 4)
        st_at(reinterpret_cast<uint4*>(snod), o + 4u * q, make_uint4(r[q], r[q + 1], r[q + 2], r[q + 3]));
    }
  }
  // SendToNeighbors (node.go:97-109): one push per out-link, draws in dest order
  const uint32_t dl = delays8<T>(x, s.draw);
  int32_t nf = 0;
#pragma unroll
  for (int k = 0; k < T::D; ++k) {
    if (k >= od) continue;  // (uniform)
    uint32_t hw = pick_hw(s, a, k);
    const uint32_t h0 = hw;
    push<T, SPILL>(x, hw, off + (uint32_t)k, on, 0x8000u | (sid << 8), s.draw + k, (dl >> (4 * k)) & 15u, s.time,
                   s.push, nf);
    const uint32_t inc = hw - h0;
#pragma unroll
    for (int v = 0; v < T::N; ++v)
      if (k < T::od(v)) s.hw[v][k] += v == a ? inc : 0u;
  }
  s.flag = nf;
  if (s.alive) s.draw += op.c;
  resolve(s);
}

// The whole event program for one wave of 64 instances (slots slot_base + wave * 64 + lane).
template <class T, bool SPILL>
__device__ __forceinline__ void program(const ExecParams& p, const Op* __restrict__ ops,
                                        const uint8_t* __restrict__ sched) {
  constexpr int N = T::N, D = T::D, RW = rec_w(T::D);
  const int32_t lane = threadIdx.x;
  const uint32_t slot = p.slot_base + blockIdx.x * (uint32_t)kWave + (uint32_t)lane;
  const bool valid = slot < (uint32_t)p.n_inst;
  const uint32_t inst = valid ? (p.inst_map ? (uint32_t)p.inst_map[slot] : slot) : 0u;
  const Layout& lay = p.lay;
  const uint32_t st = (uint32_t)p.stride;
  constexpr uint32_t capl = T::CAPL;
  const uint32_t nd = (uint32_t)(p.sched_row / 8);  // delay words (8 nibbles each)
  // 16-bit FIFO elements: lanes 0-31 in the low halves of dwords 0-31, lanes 32-63 in the high
  // halves, so each 32-lane half of a wave access hits 32 distinct banks (lane * 2 put two lanes
  // on every bank: 31M LDS bank-conflict cycles per C3 launch; 1.725 -> 1.712 ms)
  const Ctx x{(uint32_t)lane * 4u,
              ((uint32_t)lane & 31u) * 4u + ((uint32_t)lane >> 5) * 2u,
              inst,
              st,
              4u * inst * (uint32_t)N * (uint32_t)RW,
              (4u * st * (uint32_t)N * (uint32_t)RW) >> 8,
              (int32_t)(p.draws < 0x7fffffffLL ? p.draws : 0x7fffffffLL),
              Lds<T>::DB + nd - 1};

  // The instance's delay row, packed to nibbles (delays are < maxDelay = 5), in the column.
  if (valid) {
    const uint4* row = reinterpret_cast<const uint4*>(sched + (size_t)inst * p.sched_row);
    for (uint32_t q = 0; q < nd / 2; ++q) {
      const uint4 b = row[q];
      auto nib = [](uint32_t w) {
        return (w & 0xfu) | ((w >> 4) & 0xf0u) | ((w >> 8) & 0xf00u) | ((w >> 12) & 0xf000u);
      };
      col_wr(x, Lds<T>::DB + 2 * q, nib(b.x) | (nib(b.y) << 16));
      col_wr(x, Lds<T>::DB + 2 * q + 1, nib(b.z) | (nib(b.w) << 16));
    }
  }

  State<T> s;
  s.flag = 0;
#pragma unroll
  for (int w = 0; w < T::SW; ++w) s.done[w] = 0;
#pragma unroll
  for (int v = 0; v < N; ++v) {
    s.tok[v] = p.lt.init_tok[v];
#pragma unroll
    for (int k = 0; k < D; ++k) s.hw[v][k] = 0;
#pragma unroll
    for (int k = 0; k < (D + 1) / 2; ++k) s.cr[v][k] = 0;
#pragma unroll
    for (int w = 0; w < T::SW; ++w) s.pd[v][w] = 0;
  }
  s.time = s.draw = s.status = 0;
  s.peek = s.push = s.ndone = 0;
  if (p.fresh) {
    // (completion ticks are stored later by this same lane: program order keeps them after)
    if (valid)
      for (int32_t sid = 0; sid < lay.s_cap; ++sid) p.snap_tick[inst * (uint32_t)lay.s_cap + sid] = -1;
  } else if (valid) {
    // resume from the node-parallel state image (cl_engine.h Layout): per node its private
    // column words and G_* registers, then the instance's completion counters
    const uint32_t* S = p.state + inst;
    const uint32_t cap = 1u << capl;
#pragma unroll
    for (int v = 0; v < N; ++v) {
      const uint32_t b = (uint32_t)v * (uint32_t)(lay.priv + G_NUM);
      for (uint32_t q = 0; q < ((uint32_t)T::od(v) << capl); ++q)
        fifo_wr(x, (T::off(v) << capl) + q, e32_to_16(S[(b + lay.w_fifo + q) * st]));
#pragma unroll
      for (int k = 0; k < D; ++k) {
        const uint32_t lw = S[(b + lay.w_lnk + k) * st];
        if (k < T::od(v)) s.hw[v][k] = ((lw >> 8) & 0x7fu) | ((lw & 0xffu) << 7);
        if (k < T::id(v)) s.cr[v][k >> 1] |= (lw >> 16) << ((k & 1) * 16);
      }
      const uint32_t* R = S + (b + lay.priv) * st;
      s.tok[v] = (int32_t)R[G_TOKENS * st];
      const uint32_t started = R[G_STARTED * st];
      uint32_t pw[T::SW];
#pragma unroll
      for (int w = 0; w < T::SW; ++w) pw[w] = 0;
      for (int32_t sid = 0; sid < lay.s_cap; ++sid) {
        if (!((started >> sid) & 1u)) continue;
        const uint32_t pend = (S[(b + lay.w_pend + (sid >> 2)) * st] >> ((sid & 3) * 8)) & 0xffu;
        const uint32_t nib = (pend == 0 && T::id(v) == 0) ? 15u : pend + 1u;
#pragma unroll
        for (int w = 0; w < T::SW; ++w) pw[w] |= (w == (sid >> 3)) ? nib << ((sid & 7) * 4) : 0u;
      }
#pragma unroll
      for (int w = 0; w < T::SW; ++w) s.pd[v][w] = pw[w];
      if (v == 0) {
        s.time = (int32_t)R[G_TIME * st];
        s.draw = (int32_t)R[G_DRAW * st];
        s.status = (int32_t)R[G_STATUS * st];
      }
      s.peek += R[G_PEEK * st];
      s.push += R[G_PUSH * st];
    }
    const uint32_t* Dn = S + (uint32_t)N * (lay.priv + G_NUM) * st;
    for (int32_t sid = 0; sid < lay.s_cap; ++sid) {
      const uint32_t f = (int32_t)Dn[sid * st] >= N ? 8u << ((sid & 7) * 4) : 0u;
#pragma unroll
      for (int w = 0; w < T::SW; ++w) s.done[w] |= (w == (sid >> 3)) ? f : 0u;
    }
    s.ndone = Dn[lay.s_cap * st];
  }
  s.alive = valid && s.status == ST_OK;
  int32_t n_started = p.n_started_before;

  // the program through the constant address space: scalar loads, so every op field is a
  // uniform SGPR value (a vector load would make the node dispatch divergent)
  typedef const __attribute__((address_space(4))) Op COp;
  COp* cops = (COp*)ops;
  for (int32_t i = p.op_begin; i < p.op_end; ++i) {
    const Op op = cops[i];
    if (op.kind == OP_SEND) {
      send_one<T, SPILL>(x, s, op);
    } else if (op.kind == OP_SENDS) {
      // a group of sends from distinct senders: one by one is the same program (cl_engine.h)
      for (int32_t q = 1; q <= op.a; ++q) send_one<T, SPILL>(x, s, (Op)cops[i + q]);
      i += op.a;
    } else if (op.kind == OP_SNAP) {
      start_snapshot<T, SPILL>(x, s, op);
      n_started++;
    } else if (op.kind == OP_TICK || op.kind == OP_DRAIN) {
      // TICK: op.a ticks.  DRAIN: tick until every started snapshot completed (at most op.a
      // ticks, else HANG), then op.b more (test_common.go:123-137).  Per lane: a lane ticks
      // while iter < until (cl_kernels.hip exec_wave).
      const bool drain = op.kind == OP_DRAIN;
      constexpr int32_t kNoUntil = 0x7fffffff;
      int32_t until = drain ? kNoUntil : op.a;
      bool anyw = drain;
      for (int32_t iter = 0;; ++iter) {
        if (anyw) {
          const bool w = until == kNoUntil;
          if (w && (!s.alive || (int32_t)s.ndone >= n_started)) {
            until = iter + op.b;
          } else if (w && iter >= op.a) {
            s.status = ST_HANG;
            s.alive = false;
            until = iter;
          }
          anyw = __ballot(until == kNoUntil) != 0;
        }
        const bool act = s.alive && iter < until;
        if (!__ballot(act)) break;
        const bool idle = tick<T, SPILL>(x, s, act);
        if (idle && !anyw) {
          // no lane picked anything: if nothing is queued anywhere in the wave either, every
          // remaining tick of this op is empty for every lane (no peek, draw or delivery; the
          // drain tail after the last delivery, all of C3's idle wave-ticks) -- add them at once
          uint32_t q = 0;
#pragma unroll
          for (int v = 0; v < N; ++v)
#pragma unroll
            for (int k = 0; k < D; ++k)
              if (k < T::od(v)) q |= s.hw[v][k] & 0x7fu;
          if (!__ballot(q != 0)) {
            if (s.alive) s.time += max(0, until - (iter + 1));
            break;
          }
        }
      }
    }
  }

  // ---- epilogue: tokens still queued, pop counts, results, state image --------------------
  if (!valid) return;
  const uint32_t cap = 1u << capl;
  int32_t inflight = 0;
  uint32_t ptok = 0, pmk = 0, queued = 0;
#pragma unroll
  for (int v = 0; v < N; ++v) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      if (k < T::id(v)) ptok += cur_get(s, v, k);
      if (k >= T::od(v)) continue;
      const uint32_t w = s.hw[v][k], cnt = w & 0x7fu, head = (w >> 7) & 0xffu;
      const uint32_t c = T::off(v) + k;
      queued += cnt;
      for (uint32_t q = 0; q < cnt && q < cap; ++q) {
        const uint32_t e = fifo_rd(x, (c << capl) + ((head + q) & (cap - 1)));
        if (!(e & 0x8000u)) inflight += (int32_t)((e >> 8) & 0x7fu);
      }
      if (cnt > cap) {
        const uint32_t om = (1u << lay.ocap_log2) - 1;
        const uint32_t h = p.ovh[c * st + inst];
        for (uint32_t q = 0; q < cnt - cap; ++q) {
          const uint32_t e = p.ovf[((c << lay.ocap_log2) + ((h + q) & om)) * st + inst];
          if (!(e & kMarkerBit)) inflight += (int32_t)(e & 0xffffu);
        }
      }
    }
    // Queue.Pop counts (sim.go:85) derived: marker pops are indeg - pending per started snapshot
#pragma unroll
    for (int w = 0; w < T::SW; ++w)
      for (uint32_t m = s.pd[v][w]; m; m &= ~(15u << (__builtin_ctz(m) & ~3u))) {
        const uint32_t nib = (m >> (__builtin_ctz(m) & ~3u)) & 15u;
        pmk += (uint32_t)T::id(v) - (nib == 15u ? 0u : nib - 1u);
      }
  }
  int32_t* r = p.regs + (size_t)inst * R_NUM;
  r[R_TIME] = s.time;
  r[R_DRAW] = s.draw;
  r[R_STATUS] = s.status;
  r[R_NDONE] = (int32_t)s.ndone;
  r[R_PEEK] = (int32_t)s.peek;
  r[R_POP_TOK] = (int32_t)ptok;
  r[R_POP_MK] = (int32_t)pmk;
  // Queue.Push count (queue.go:18-20) derived like the pops: every packet pushed since the
  // program's start was either popped or is still queued (LDS ring or HBM spill ring)
  const uint32_t pushes = ptok + pmk + queued;
  r[R_PUSH] = (int32_t)pushes;
  r[R_INFLIGHT_TOK] = inflight;
#pragma unroll
  for (int v = 0; v < N; ++v) p.fin_tok[inst * (uint32_t)N + v] = s.tok[v];
  if (!p.save_state) return;
  // the node-parallel state image (peek and push counts as node 0's, the others 0)
  uint32_t* S = p.state + inst;
#pragma unroll
  for (int v = 0; v < N; ++v) {
    const uint32_t b = (uint32_t)v * (uint32_t)(lay.priv + G_NUM);
    for (int32_t k = 0; k < lay.priv; ++k) S[(b + k) * st] = 0u;
    for (uint32_t q = 0; q < ((uint32_t)T::od(v) << capl); ++q)
      S[(b + lay.w_fifo + q) * st] = e16_to_32(fifo_rd(x, (T::off(v) << capl) + q), s.time);
#pragma unroll
    for (int k = 0; k < D; ++k) {
      uint32_t lw = k < T::id(v) ? cur_get(s, v, k) << 16 : 0u;
      if (k < T::od(v)) {
        const uint32_t w = s.hw[v][k];
        lw |= ((w >> 7) & (cap - 1)) | ((w & 0x7fu) << 8);
      }
      S[(b + lay.w_lnk + k) * st] = lw;
    }
    uint32_t started = 0;
    for (int32_t sid = 0; sid < lay.s_cap; ++sid) {
      uint32_t pw = 0;
#pragma unroll
      for (int w = 0; w < T::SW; ++w) pw = (w == (sid >> 3)) ? s.pd[v][w] : pw;
      const uint32_t nib = (pw >> ((sid & 7) * 4)) & 15u;
      if (!nib) continue;
      started |= 1u << sid;
      const uint32_t pend = nib == 15u ? 0u : nib - 1u;
      S[(b + lay.w_pend + (sid >> 2)) * st] |= pend << ((sid & 3) * 8);
    }
    uint32_t* R = S + (b + lay.priv) * st;
    R[G_TOKENS * st] = (uint32_t)s.tok[v];
    R[G_STARTED * st] = started;
    R[G_TIME * st] = (uint32_t)s.time;
    R[G_DRAW * st] = (uint32_t)s.draw;
    R[G_STATUS * st] = (uint32_t)s.status;
    R[G_PEEK * st] = v == 0 ? s.peek : 0u;
    R[G_POP_TOK * st] = v == 0 ? ptok : 0u;  // (informational: a continuation derives them again)
    R[G_POP_MK * st] = v == 0 ? pmk : 0u;
    R[G_PUSH * st] = v == 0 ? pushes : 0u;
  }
  uint32_t* Dn = S + (uint32_t)N * (lay.priv + G_NUM) * st;
  for (int32_t sid = 0; sid < lay.s_cap; ++sid) {
    uint32_t c = 0;
#pragma unroll
    for (int v = 0; v < N; ++v) {
      uint32_t pw = 0;
#pragma unroll
      for (int w = 0; w < T::SW; ++w) pw = (w == (sid >> 3)) ? s.pd[v][w] : pw;
      c += ((pw >> ((sid & 7) * 4)) & 15u) == 1u ? 1u : 0u;
    }
    Dn[sid * st] = c;
  }
  Dn[lay.s_cap * st] = s.ndone;
}

}  // namespace lanes
}  // namespace clsnap
