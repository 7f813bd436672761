// cl_host.cpp -- host runtime behind include/clsnap.h.
//
// The host side mirrors the reference's Simulator API (sim.go, node.go) and its
// drivers (test_common.go) over a batch of instances:
//   * topology: AddNode/AddLink collected, then frozen into rank order (getSortedKeys,
//     common.go:135-146) as out-CSR (channels by (src rank, dest rank)) and in-CSR;
//   * events: SendTokens / StartSnapshot / Tick / drain become an op program that the
//     gfx950 kernel executes for every instance (cl_kernels.hip);
//   * delays: the reference's rand.Intn(5) (sim.go:101) is replayed from a per-instance
//     schedule, by default Go's own math/rand stream for seed_base + i, restated here;
//   * results: snapshots are packed back into the reference's {tokenMap, messages}
//     shape (sim.go:134-173) per instance.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/clsnap.h"
#include "cl_engine.h"
#include "cl_text.h"

using namespace clsnap;

namespace clsnap {
namespace {
thread_local std::string g_last_error;
}
int set_error_v(int code, const char* fmt, va_list ap) {
  char buf[512];
  vsnprintf(buf, sizeof buf, fmt, ap);
  g_last_error = buf;
  return code;
}
const char* last_error() { return g_last_error.c_str(); }
}  // namespace clsnap

// Per-wave LDS words available for staging the wave's delay rows (kernel reads the
// delays from LDS instead of HBM when ipw * row fits).
constexpr int32_t kDelayStageWords = 2048;
// Workgroups (4 waves each) per CU the automatic FIFO sizing keeps LDS from limiting (the
// spill-free kernels of degree bounds 3-4 run 6 waves per SIMD; deeper queues spill to HBM).
constexpr int32_t kTargetBlocks = 6;
// Batches of at least this many instances replay through a length-ordered slot map (a few
// thousand waves: the grouping pays for its one host sort and 4 B per instance of HBM).
constexpr int64_t kMapMinInstances = 4096;

// A length-ordered slot map is used when it keeps at most this % of the wave-ticks of the
// unordered launch (C3 90 %: kept; C2 95 %: measured slower mapped, §9)
constexpr int64_t kMapPct = 92;

namespace {

int set_err(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  const int rc = set_error_v(code, fmt, ap);
  va_end(ap);
  return rc;
}

// ---------------------------------------------------------------------------
// Go math/rand (Go 1.22, go.mod:3): rngSource seeded as in rng.go, Intn -> Int31n.
// rngCooked is regenerated offline by oracle/gen_go_rng_cooked.py (KAT-pinned).
// ---------------------------------------------------------------------------
const int64_t kRngCooked[607] = {
#include "go_rng_cooked.inc"
};

struct GoRand {
  int tap = 0, feed = 334;
  uint64_t vec[607];

  static int32_t seedrand(int32_t x) {
    const int32_t hi = x / 44488, lo = x % 44488;
    x = 48271 * lo - 3399 * hi;
    if (x < 0) x += 2147483647;
    return x;
  }
  explicit GoRand(int64_t seed) {
    seed %= 2147483647LL;
    if (seed < 0) seed += 2147483647LL;
    if (seed == 0) seed = 89482311;
    int32_t x = (int32_t)seed;
    for (int i = -20; i < 607; ++i) {
      x = seedrand(x);
      if (i >= 0) {
        uint64_t u = (uint64_t)(int64_t)x << 40;
        x = seedrand(x);
        u ^= (uint64_t)(int64_t)x << 20;
        x = seedrand(x);
        u ^= (uint64_t)(int64_t)x;
        vec[i] = u ^ (uint64_t)kRngCooked[i];
      }
    }
  }
  uint64_t uint64() {
    if (--tap < 0) tap += 607;
    if (--feed < 0) feed += 607;
    vec[feed] += vec[tap];
    return vec[feed];
  }
  int64_t int63() { return (int64_t)(uint64() & 0x7fffffffffffffffULL); }
  int32_t int31() { return (int32_t)(int63() >> 32); }
  int32_t int31n(int32_t n) {
    if ((n & (n - 1)) == 0) return int31() & (n - 1);
    const int32_t max = (int32_t)((1LL << 31) - 1 - (int64_t)((1ULL << 31) % (uint32_t)n));
    int32_t v = int31();
    while (v > max) v = int31();
    return v % n;
  }
};

int host_threads() {
  unsigned n = std::thread::hardware_concurrency();
  if (n == 0) n = 1;
  return (int)std::min(n, 16u);  // the GPU box grants 16 host cores per GPU
}

void go_schedule(int64_t seed_base, int64_t n, int64_t draws, uint8_t* out) {
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(host_threads(), (n + 255) / 256));
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) {
    th.emplace_back([=] {
      for (int64_t i = n * t / T; i < n * (t + 1) / T; ++i) {
        GoRand r(seed_base + i);
        uint8_t* o = out + i * draws;
        for (int64_t k = 0; k < draws; ++k) o[k] = (uint8_t)r.int31n(5);  // rand.Intn(maxDelay)
      }
    });
  }
  for (auto& x : th) x.join();
}

#define HIP_TRY(expr)                                                                     \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess) return set_err(CL_E_DEVICE, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  int ensure(size_t count) {
    if (count <= n && p) return CL_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    if (count == 0) count = 1;
    HIP_TRY(hipMalloc((void**)&p, count * sizeof(T)));
    n = count;
    return CL_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

}  // namespace

// ---------------------------------------------------------------------------
// cl_sim
// ---------------------------------------------------------------------------
struct cl_sim {
  // Every ABI call on a sim holds `mu` (recursive: the drivers call the event entry
  // points).  A collector thread may poll / wait / collect while the driver thread
  // issues events and ticks (sim.go:134-173 runs CollectSnapshot on its own goroutine,
  // test_common.go:106-108); `executed_cv` is signalled after every execution.
  mutable std::recursive_mutex mu;
  std::condition_variable_any executed_cv;
  uint64_t exec_gen = 0;  // executions completed (flushes that ran ops) and ticks issued
  int32_t waiters = 0;    // threads blocked in cl_wait_snapshot
  bool closing = false;   // cl_sim_destroy has begun: waiters leave with CL_E_STATE

  // A tick or drain was issued: a waiter re-checks (its check executes the pending events),
  // so a driver that only calls Tick() -- the reference pattern -- still wakes a blocked
  // CollectSnapshot (sim.go:137-140).
  void notify_waiters() {
    if (!waiters) return;
    ++exec_gen;
    executed_cv.notify_all();
  }

  int64_t n_inst = 0;
  int64_t stride = 0;  // n_inst rounded up to the wave size
  int device = 0;

  // topology (insertion order until frozen)
  std::vector<std::string> ids;
  std::vector<int64_t> init_tokens;
  std::unordered_map<std::string, int> id_index;
  std::vector<std::pair<int, int>> links;  // unique (src, dst) in insertion indices
  bool frozen = false;
  std::vector<int> rank_of;    // insertion index -> rank
  std::vector<int> by_rank;    // rank -> insertion index
  std::vector<int32_t> out_off, ch_dst, ch_src, in_off, in_ch, init_tok;
  int32_t max_out = 0, max_in = 0;
  int64_t total_tokens = 0;

  // event program
  std::vector<Op> ops;
  int32_t executed = 0;
  int32_t n_sids = 0;
  int64_t sends = 0;
  int64_t time_bound = 0;
  std::vector<std::vector<int32_t>> hist;  // token history per channel (push order)
  std::vector<int32_t> depth_bound;        // packets ever pushed per channel

  // exec kernel choice (cl_set_exec_engine) and the one the latest launch used
  int32_t engine = CL_ENGINE_AUTO;
  int32_t last_engine = 0;

  // limits
  int32_t cap_log2 = 3;
  bool auto_cap = true;  // choose cap_log2 per layout (cl_set_limits with slots > 0 pins it)
  int64_t max_drain = 10000;

  // delays
  bool go_seeds = true;
  int64_t seed_base = 8053172852482175524LL;  // snapshot_test.go:9,20 (seed + 1)
  std::vector<uint8_t> user_sched;
  int64_t user_draws = 0;
  int64_t dev_draws = -1;  // valid draws per instance of the schedule resident on the device
  int64_t dev_row = 0;     // its row stride (multiple of 16)

  // device
  bool dev_ready = false;
  hipStream_t stream = nullptr;
  bool timed = false;
  // per-launch timing events: start, stop, and the split replay's spill-capable start / stop
  // (the launch time is the longer of the two concurrent halves: consecutive replays are not
  // joined, so a half's own events, not the other stream's, bound it)
  struct LaunchEvents {
    hipEvent_t start = nullptr, stop = nullptr, start2 = nullptr, stop2 = nullptr;
    int32_t stop2_used = 0;
  };
  std::vector<LaunchEvents> ev_pool;
  size_t ev_used = 0;
  double ev_folded_ms = 0;   // time of launches whose events were recycled
  int64_t ev_folded_n = 0;
  size_t ev_last = 0;        // pool entry of the latest launch (cl_last_kernel_ms)

  int launch_ms(const LaunchEvents& e, float* ms) const {
    HIP_TRY(hipEventElapsedTime(ms, e.start, e.stop));
    if (e.stop2_used) {
      float f2 = 0.f;
      HIP_TRY(hipEventElapsedTime(&f2, e.start2, e.stop2));
      *ms = std::max(*ms, f2);
    }
    return CL_OK;
  }

  // Fold finished launch timings into the accumulator so the event pool stays bounded.
  int fold_events() {
    HIP_TRY(hipStreamSynchronize(stream));
    // (a pipelined replay's spill-capable stop event is recorded on stream2, which `stream` may
    // not have joined yet: cl_rerun folds every 256 launches without a join)
    if (stream2) HIP_TRY(hipStreamSynchronize(stream2));
    for (size_t i = 0; i < ev_used; ++i) {
      float f = 0.f;
      int rc = launch_ms(ev_pool[i], &f);
      if (rc) return rc;
      ev_folded_ms += f;
    }
    ev_folded_n += (int64_t)ev_used;
    if (ev_used) std::swap(ev_pool[0], ev_pool[ev_used - 1]);
    ev_last = 0;
    ev_used = 0;
    return CL_OK;
  }
  Layout lay{};
  int32_t s_cap = 0;
  bool need_fresh = true;
  bool state_valid = false;  // the device state image matches ops[0, executed)
  int64_t layout_row = 0;    // delay row length the LDS layout was sized for
  DevBuf<Op> d_ops;
  // Device program: `ops` with runs of sends from distinct senders folded into OP_SENDS
  // groups; dmap[i] = device index of logical op i (every launch begins at a group start).
  std::vector<Op> dops;
  std::vector<int32_t> dmap;
  size_t dops_for = 0;
  int32_t dops_begin = -1;
  DevBuf<uint32_t> d_topo;
  DevBuf<int32_t> d_fin_tok;
  DevBuf<uint8_t> d_sched;
  DevBuf<uint32_t> d_state;
  DevBuf<int32_t> d_regs;
  DevBuf<uint32_t> d_snap_nod;  // [s_cap][stride][n][lay.rw] node snapshot records
  DevBuf<int32_t> d_ch_slot;    // [C] word of channel c in an instance's records
  DevBuf<int32_t> d_snap_tick;
  DevBuf<uint32_t> d_ovf;
  DevBuf<uint32_t> d_ovh;
  // Replay plan (build_plan), from the first fresh full run of ops [0, plan_ops) with these
  // delays and layout -- the probe, run on the spill-capable kernel with per-instance spill
  // flags.  Its replays (cl_rerun: the same program and delays, hence the same queues and
  // final ticks) launch through a slot map d_map: instances grouped by their final tick so the
  // 64 / N instances sharing a wave end their drains together, and the instances that spilled
  // last; slots [0, split_slot) then run the spill-free kernel (6 waves per SIMD at degree
  // bounds 3-4) and the rest the spill-capable one, concurrently on stream2.  Results are per
  // instance and identical on either kernel.
  DevBuf<uint8_t> d_spill_inst;  // [n_inst] probe: 1 where a push spilled to HBM
  int64_t plan_ops = -1;         // program length the plan holds for (-1: none)
  int64_t plan_tried = -1;       // program length a probe last ran for
  bool probe = false;            // the last launch was a probe (plan built at the next sync)
  int64_t probe_ops = 0;
  bool probe_flags = false;      // the probe recorded spill flags
  bool plan_map = false, plan_nospill = false;
  int64_t plan_split = 0, plan_spilled = 0;
  hipStream_t stream2 = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // Split replays back to back: the spill-capable half of a replay on stream2
  // and the spill-free half on `stream` touch disjoint instances, so consecutive replays need
  // no cross-stream wait between them -- a replay's halves overlap the previous replay's
  // tail.  s2_live: stream2 may hold work `stream` has not waited for; every other ABI call
  // joins it first (join_stream2, SIM_CHECK).  s_dirty: `stream` got work since the last
  // fork, so the next replay's stream2 half must wait for it.
  bool s2_live = false, s_dirty = true;
  int join_stream2() {
    s_dirty = true;
    if (!s2_live) return CL_OK;
    s2_live = false;
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipEventRecord(ev_join, stream2));
    HIP_TRY(hipStreamWaitEvent(stream, ev_join, 0));
    return CL_OK;
  }
  // wave end their drains together; replays of the same program and delays launch through
  // the map (results are per instance, unchanged).  -1: no map.
  DevBuf<int32_t> d_map;
  DevBuf<int32_t> d_hist;
  DevBuf<unsigned long long> d_sums;
  // device event trace (cl_trace_enable): instances [trace_lo, trace_lo + trace_n)
  DevBuf<TraceRec> d_trace;
  DevBuf<uint32_t> d_trace_cnt;
  DevBuf<int32_t> d_ch_dest;
  int64_t trace_lo = 0;
  int32_t trace_n = 0, trace_cap = 0;

  // host mirrors of the per-instance results (invalidated by every launch); the snapshot
  // records stay on the device: collects pack them there (cl_pack_*), a one-instance collect
  // copies that instance's records only
  bool h_valid = false;
  std::vector<int32_t> h_regs, h_snap_tick, h_tok, ch_slot;
  // device-side CollectSnapshot packing (PackParams)
  DevBuf<int32_t> d_pk_tok, d_pk_done, d_pk_msg;
  DevBuf<long long> d_pk_cnt, d_pk_bsum, d_pk_off;
  DevBuf<unsigned long long> d_rec2;
  hipEvent_t pk_ev[2] = {nullptr, nullptr};
  bool pk_timed = false;
  size_t hist_uploaded = (size_t)-1;  // history entries on the device

  ~cl_sim() {
    if (dev_ready) {
      (void)hipSetDevice(device);
      if (stream2) (void)hipStreamSynchronize(stream2);
      (void)hipStreamSynchronize(stream);
      d_ops.release(); d_topo.release(); d_sched.release(); d_state.release(); d_regs.release();
      d_snap_nod.release(); d_ch_slot.release(); d_snap_tick.release(); d_ovf.release(); d_fin_tok.release();
      d_ovh.release(); d_spill_inst.release(); d_map.release(); d_hist.release(); d_sums.release();
      d_trace.release(); d_trace_cnt.release(); d_ch_dest.release();
      d_pk_tok.release(); d_pk_done.release(); d_pk_msg.release(); d_pk_cnt.release(); d_pk_bsum.release();
      d_pk_off.release(); d_rec2.release();
      for (auto& e : pk_ev)
        if (e) (void)hipEventDestroy(e);
      for (auto& e : ev_pool) {
        (void)hipEventDestroy(e.start);
        (void)hipEventDestroy(e.stop);
        (void)hipEventDestroy(e.stop2);
        (void)hipEventDestroy(e.start2);
      }
      if (stream2) (void)hipStreamDestroy(stream2);
      if (ev_fork) (void)hipEventDestroy(ev_fork);
      if (ev_join) (void)hipEventDestroy(ev_join);
      (void)hipStreamDestroy(stream);
    }
  }

  int node_of(const char* id) const {
    auto it = id_index.find(id ? std::string(id) : std::string());
    return it == id_index.end() ? -1 : it->second;
  }

  // Freeze the topology into rank order (getSortedKeys, common.go:135-146).
  int freeze() {
    if (frozen) return CL_OK;
    const int n = (int)ids.size();
    if (n > kMaxNodes) return set_err(CL_E_LIMIT, "%d nodes exceed the node-parallel engine limit %d", n, kMaxNodes);
    by_rank.resize(n);
    for (int i = 0; i < n; ++i) by_rank[i] = i;
    std::sort(by_rank.begin(), by_rank.end(), [&](int a, int b) { return ids[a] < ids[b]; });
    rank_of.assign(n, 0);
    for (int r = 0; r < n; ++r) rank_of[by_rank[r]] = r;
    std::vector<std::pair<int, int>> ch;
    for (auto& l : links) ch.emplace_back(rank_of[l.first], rank_of[l.second]);
    std::sort(ch.begin(), ch.end());
    const int C = (int)ch.size();
    out_off.assign(n + 1, 0);
    in_off.assign(n + 1, 0);
    ch_dst.resize(C);
    ch_src.resize(C);
    for (int c = 0; c < C; ++c) {
      ch_src[c] = ch[c].first;
      ch_dst[c] = ch[c].second;
      out_off[ch[c].first + 1]++;
      in_off[ch[c].second + 1]++;
    }
    for (int v = 0; v < n; ++v) {
      out_off[v + 1] += out_off[v];
      in_off[v + 1] += in_off[v];
    }
    in_ch.resize(C);
    std::vector<int32_t> fill(in_off.begin(), in_off.end() - 1);
    for (int c = 0; c < C; ++c) in_ch[fill[ch_dst[c]]++] = c;  // channels sorted by src: in-lists by src rank
    init_tok.resize(n);
    total_tokens = 0;
    for (int r = 0; r < n; ++r) {
      init_tok[r] = (int32_t)init_tokens[by_rank[r]];
      total_tokens += init_tokens[by_rank[r]];
    }
    max_out = max_in = 0;
    for (int v = 0; v < n; ++v) {
      max_out = std::max(max_out, out_off[v + 1] - out_off[v]);
      max_in = std::max(max_in, in_off[v + 1] - in_off[v]);
    }
    if (max_out > kMaxDegree) return set_err(CL_E_LIMIT, "out-degree %d exceeds %d", max_out, kMaxDegree);
    hist.assign(C, {});
    depth_bound.assign(C, 0);
    frozen = true;
    return CL_OK;
  }

  int channel_of(int src_rank, int dst_rank) const {
    for (int c = out_off[src_rank]; c < out_off[src_rank + 1]; ++c)
      if (ch_dst[c] == dst_rank) return c;
    return -1;
  }

  int64_t draws_needed() const { return sends + (int64_t)n_sids * (int64_t)ch_dst.size(); }

  int ocap_log2_needed() const {
    int32_t mx = 0;
    for (auto d : depth_bound) mx = std::max(mx, d);
    const int32_t cap = 1 << cap_log2;
    if (mx <= cap) return -1;
    int need = std::min(mx, kMaxQueued) - cap, l = 0;
    while ((1 << l) < need) ++l;
    return l;
  }

  int ensure_device() {
    if (dev_ready) return CL_OK;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
      return set_err(CL_E_DEVICE, "no HIP device available (the engine needs a gfx950 GPU)");
    if (device < 0 || device >= count) return set_err(CL_E_DEVICE, "device %d out of range (%d)", device, count);
    HIP_TRY(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
      return set_err(CL_E_DEVICE, "device %d is %s, the engine is built for gfx950", device, prop.gcnArchName);
    HIP_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    dev_ready = true;
    return CL_OK;
  }

  int upload_topology() {
    const int n = (int)ids.size();
    const int W = 3 + max_in;
    std::vector<uint32_t> t((size_t)n * W + n, 0u);
    for (int v = 0; v < n; ++v) {
      uint32_t* b = &t[(size_t)v * W];
      b[0] = (uint32_t)(in_off[v + 1] - in_off[v]);
      b[1] = (uint32_t)(out_off[v + 1] - out_off[v]);
      b[2] = (uint32_t)out_off[v];
      for (int k = in_off[v]; k < in_off[v + 1]; ++k) {
        const int c = in_ch[k], src = ch_src[c];
        b[3 + (k - in_off[v])] = (uint32_t)src | ((uint32_t)(c - out_off[src]) << 8) | ((uint32_t)c << 16);
      }
      t[(size_t)n * W + v] = (uint32_t)init_tok[v];
    }
    int rc = d_topo.ensure(t.size());
    if (rc) return rc;
    HIP_TRY(hipMemcpy(d_topo.p, t.data(), t.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    if ((rc = d_ch_dest.ensure(std::max<size_t>(ch_dst.size(), 1)))) return rc;
    if (!ch_dst.empty())
      HIP_TRY(hipMemcpy(d_ch_dest.p, ch_dst.data(), ch_dst.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    return CL_OK;
  }

  int ensure_delays() {
    int64_t need = draws_needed();
    if (go_seeds) {
      int64_t D = std::max<int64_t>(16, (need + 15) / 16 * 16);
      if (dev_draws >= D) return CL_OK;
      std::vector<uint8_t> sched((size_t)(D * n_inst));
      go_schedule(seed_base, n_inst, D, sched.data());
      if (dev_ready) HIP_TRY(hipStreamSynchronize(stream));  // (an async launch may read d_sched)
      int rc = d_sched.ensure(sched.size());
      if (rc) return rc;
      HIP_TRY(hipMemcpy(d_sched.p, sched.data(), sched.size(), hipMemcpyHostToDevice));
      dev_draws = D;  // longer rows of the same streams: saved draw cursors stay valid
      plan_ops = plan_tried = -1;
      dev_row = D;
      return CL_OK;
    }
    if (dev_draws == user_draws) return CL_OK;
    const int64_t row = (user_draws + 15) / 16 * 16;
    std::vector<uint8_t> padded((size_t)(row * n_inst), 0);
    for (int64_t i = 0; i < n_inst; ++i)
      std::memcpy(&padded[(size_t)(i * row)], &user_sched[(size_t)(i * user_draws)], (size_t)user_draws);
    if (dev_ready) HIP_TRY(hipStreamSynchronize(stream));  // (an async launch may read d_sched)
    int rc = d_sched.ensure(padded.size());
    if (rc) return rc;
    HIP_TRY(hipMemcpy(d_sched.p, padded.data(), padded.size(), hipMemcpyHostToDevice));
    dev_draws = user_draws;
    dev_row = row;
    plan_ops = plan_tried = -1;
    return CL_OK;
  }

  // The layout the next launch would use: s_cap, the LDS ring size and the delay row (no
  // allocation; ensure_layout applies it).
  Layout plan_layout(int32_t* s_cap_out, int32_t* cap_log2_out, int64_t* row_out) const {
    const int n = (int)ids.size();
    const int32_t want_s = std::max<int32_t>(4, (n_sids + 3) / 4 * 4);
    const int32_t sc = std::max(want_s, s_cap);
    const int64_t row = go_seeds ? std::max<int64_t>(16, (draws_needed() + 15) / 16 * 16) : (user_draws + 15) / 16 * 16;
    const int32_t od = std::max(max_out, 1), id = std::max(max_in, 1);
    int32_t cl = cap_log2;
    if (auto_cap) {
      // LDS ring slots per channel: enough for the deepest channel (spill beyond), but
      // small enough that LDS does not cap the workgroups per CU below kTargetBlocks.
      int32_t mx = 1;
      for (auto d : depth_bound) mx = std::max(mx, d);
      int l = 1;
      while (l < 3 && (1 << l) < mx) ++l;  // at most 8 slots
      for (; l > 1; --l) {
        Layout t = make_layout(n, od, id, l, -1, sc, row, kDelayStageWords);
        if ((int64_t)t.wave_words * kWavesPerBlock * 4 * kTargetBlocks <= kMaxLdsBytes) break;
      }
      cl = l;
    }
    int32_t mx = 0;
    for (auto d : depth_bound) mx = std::max(mx, d);
    int ocap = -1;
    if (mx > (1 << cl)) {
      int need = std::min(mx, kMaxQueued) - (1 << cl), l = 0;
      while ((1 << l) < need) ++l;
      ocap = l;
    }
    if (s_cap_out) *s_cap_out = sc;
    if (cap_log2_out) *cap_log2_out = cl;
    if (row_out) *row_out = row;
    return make_layout(n, od, id, cl, std::max(ocap, lay.wave_words ? lay.ocap_log2 : -1), sc, row, kDelayStageWords);
  }

  // Allocate per-instance state and outputs for the current layout.
  int ensure_layout() {
    const int n = (int)ids.size(), C = (int)ch_dst.size();
    int32_t want_s = std::max<int32_t>(4, (n_sids + 3) / 4 * 4);
    int ocap = ocap_log2_needed();
    if (!need_fresh && lay.wave_words && want_s <= s_cap && ocap <= lay.ocap_log2 && lay.cap_log2 == cap_log2 &&
        layout_row == (go_seeds ? std::max<int64_t>(16, (draws_needed() + 15) / 16 * 16) : (user_draws + 15) / 16 * 16))
      return CL_OK;
    if (dev_ready) HIP_TRY(hipStreamSynchronize(stream));  // (buffers below may be reallocated or rewritten)
    if (n == 0) return set_err(CL_E_STATE, "the topology has no nodes");
    int64_t row = 0;
    int32_t sc = 0, cl = 0;
    Layout L = plan_layout(&sc, &cl, &row);
    s_cap = sc;
    cap_log2 = cl;
    if (s_cap > kMaxSnapshots) return set_err(CL_E_LIMIT, "more than %d snapshots", kMaxSnapshots);
    if (4ull * s_cap * stride * (uint64_t)n * (uint64_t)L.rw >= (1ull << 32) ||  // byte offsets
        (uint64_t)L.state_words * stride >= (1ull << 32))
      return set_err(CL_E_LIMIT, "batch too large for 32-bit output indexing; split it");
    // high-degree topologies: fewer waves per workgroup (one wave's state must fit)
    while (L.wpb > 1 && (int64_t)L.wave_words * L.wpb * 4 > kMaxLdsBytes) L.wpb /= 2;
    if ((int64_t)L.wave_words * L.wpb * 4 > kMaxLdsBytes)
      return set_err(CL_E_LIMIT, "per-wave state of %d words exceeds LDS (lower fifo slots or degree)", L.wave_words);
    lay = L;
    layout_row = row;
    int rc;
    if ((rc = d_state.ensure((size_t)lay.state_words * stride))) return rc;
    if ((rc = d_regs.ensure((size_t)R_NUM * stride))) return rc;
    if ((rc = d_fin_tok.ensure((size_t)n * stride))) return rc;
    if ((rc = d_snap_nod.ensure((size_t)s_cap * n * lay.rw * stride))) return rc;
    ch_slot.assign(std::max(C, 1), 0);
    for (int v = 0; v < n; ++v)
      for (int k = in_off[v]; k < in_off[v + 1]; ++k) ch_slot[in_ch[k]] = v * lay.rw + 1 + (k - in_off[v]);
    if ((rc = d_ch_slot.ensure(ch_slot.size()))) return rc;
    HIP_TRY(hipMemcpy(d_ch_slot.p, ch_slot.data(), ch_slot.size() * 4, hipMemcpyHostToDevice));
    if ((rc = d_snap_tick.ensure((size_t)s_cap * stride))) return rc;
    const size_t ov = lay.ocap_log2 >= 0 ? ((size_t)C << lay.ocap_log2) * stride : 1;
    if ((rc = d_ovf.ensure(ov))) return rc;
    if ((rc = d_ovh.ensure(lay.ocap_log2 >= 0 ? (size_t)std::max(C, 1) * stride : 1))) return rc;
    if (lay.ocap_log2 >= 0 && (rc = d_spill_inst.ensure((size_t)n_inst))) return rc;
    plan_ops = plan_tried = -1;
    need_fresh = true;
    return CL_OK;
  }

  int upload_hist() {
    size_t tot = 0;
    for (auto& h : hist) tot += h.size();
    if (tot == hist_uploaded && d_hist.p) return CL_OK;  // (histories only grow: same size, same data)
    hist_uploaded = tot;
    std::vector<int32_t> off(1, 0), val;
    for (auto& h : hist) {
      val.insert(val.end(), h.begin(), h.end());
      off.push_back((int32_t)val.size());
    }
    std::vector<int32_t> all(off);
    all.insert(all.end(), val.begin(), val.end());
    int rc = d_hist.ensure(all.size());
    if (rc) return rc;
    HIP_TRY(hipMemcpy(d_hist.p, all.data(), all.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    return CL_OK;
  }

  // Fold every maximal run of consecutive sends with pairwise distinct senders (and not
  // crossing the launch start `begin`) into one OP_SENDS group.  Within such a run no send
  // changes another's sender balance or channel, so the kernel can run them in parallel
  // lanes with draw k + position (the reference's draw order, sim.go:101).
  void build_device_program(int32_t begin) {
    dops.clear();
    dmap.assign(ops.size() + 1, 0);
    size_t i = 0;
    while (i < ops.size()) {
      size_t j = i + 1;
      if (ops[i].kind == OP_SEND) {
        uint64_t seen = 1ull << ops[i].a;
        while (j < ops.size() && ops[j].kind == OP_SEND && (int64_t)j != begin && !((seen >> ops[j].a) & 1ull)) {
          seen |= 1ull << ops[j].a;
          ++j;
        }
      }
      if (j - i >= 2) {
        for (size_t k = i; k < j; ++k) dmap[k] = (int32_t)dops.size();
        dops.push_back(Op{OP_SENDS, (int32_t)(j - i), 0, 0});
        dops.insert(dops.end(), ops.begin() + i, ops.begin() + j);
      } else {
        dmap[i] = (int32_t)dops.size();
        dops.push_back(ops[i]);
      }
      i = j;
    }
    dmap[ops.size()] = (int32_t)dops.size();
  }

  // The frozen topology in the form the instance-per-lane kernels are generated from (cl_jit.cpp):
  // ok only for N <= 16 nodes with every degree <= 4.
  LanesTopo lanes_topo() const {
    LanesTopo t{};
    const int n = (int)ids.size();
    if (n < 1 || n > kLanesMaxNodes || max_out > kLanesMaxDegree || max_in > kLanesMaxDegree) return t;
    for (int v = 0; v < n; ++v) {
      const int id = in_off[v + 1] - in_off[v], od = out_off[v + 1] - out_off[v];
      t.node[v] = (uint32_t)id | ((uint32_t)od << 4) | ((uint32_t)out_off[v] << 8);
      for (int j = 0; j < id; ++j) {
        const int c = in_ch[in_off[v] + j], src = ch_src[c];
        t.inl[v] |= ((uint32_t)src | ((uint32_t)(c - out_off[src]) << 4)) << (8 * j);
      }
      t.init_tok[v] = init_tok[v];
    }
    t.ok = out_off[n] <= 255 ? 1 : 0;
    for (const Op& o : ops)
      if (o.kind == OP_SEND) t.max_payload = std::max(t.max_payload, o.c);
    for (auto d : depth_bound) t.max_depth = std::max(t.max_depth, d);
    return t;
  }

  ExecParams exec_params(int32_t op_begin, int32_t n_started_before) const {
    ExecParams p{};
    const int n = (int)ids.size(), C = (int)ch_dst.size();
    p.op_begin = dmap[op_begin];
    p.op_end = (int32_t)dops.size();
    p.n_nodes = n;
    p.n_ch = C;
    p.lay = lay;
    p.n_started_before = n_started_before;
    p.topo_w = 3 + max_in;  // ensure_layout guarantees lay.od == lay.id >= every node's degree
    p.draws = dev_draws;
    p.sched_row = dev_row;
    p.n_inst = n_inst;
    p.stride = stride;
    p.fresh = op_begin == 0 ? 1 : 0;
    p.state = d_state.p;
    p.regs = d_regs.p;
    p.fin_tok = d_fin_tok.p;
    p.snap_nod = d_snap_nod.p;
    p.snap_tick = d_snap_tick.p;
    p.ovf = d_ovf.p;
    p.ovh = d_ovh.p;
    p.ch_dest = d_ch_dest.p;
    p.lt = lanes_topo();
    if (trace_n > 0) {
      p.trace = d_trace.p;
      p.trace_cnt = d_trace_cnt.p;
      p.trace_lo = trace_lo;
      p.trace_n = trace_n;
      p.trace_cap = trace_cap;
    }
    return p;
  }

  // Launch pending ops (all ops when a fresh replay is needed). Asynchronous.
  int launch(bool force_fresh, bool save_state) {
    int rc = freeze();
    if (rc) return rc;
    if ((rc = ensure_device())) return rc;
    HIP_TRY(hipSetDevice(device));
    if (!d_topo.p && (rc = upload_topology())) return rc;
    if ((rc = ensure_layout())) return rc;
    if ((rc = ensure_delays())) return rc;
    if (lay.x_delay && dev_row != layout_row)
      return set_err(CL_E_STATE, "delay rows (%lld) differ from the staged layout (%lld)", (long long)dev_row,
                     (long long)layout_row);
    if (force_fresh || !state_valid) need_fresh = true;
    if (!need_fresh && executed == (int32_t)ops.size()) return CL_OK;
    int32_t begin = need_fresh ? 0 : executed;
    if (ops.size() != dops_for || begin != dops_begin || !d_ops.p) {
      build_device_program(begin);
      // an earlier asynchronous launch (cl_rerun) may still read d_ops: a null-stream copy
      // does not wait for the engine's non-blocking stream
      HIP_TRY(hipStreamSynchronize(stream));
      if ((rc = d_ops.ensure(std::max<size_t>(dops.size(), 64)))) return rc;
      HIP_TRY(hipMemcpy(d_ops.p, dops.data(), dops.size() * sizeof(Op), hipMemcpyHostToDevice));
      dops_for = ops.size();
      dops_begin = begin;
    }
    int32_t started_before = 0;
    for (int32_t i = 0; i < begin; ++i) started_before += ops[i].kind == OP_SNAP;
    if (trace_n > 0) {
      if ((rc = d_trace.ensure((size_t)trace_n * trace_cap)) || (rc = d_trace_cnt.ensure((size_t)trace_n))) return rc;
      // a replay from the initial state restarts the log (a resumed launch appends)
      if (begin == 0) HIP_TRY(hipMemsetAsync(d_trace_cnt.p, 0, (size_t)trace_n * sizeof(uint32_t), stream));
    }
    // (a fresh replay's kernel sets snap_tick to -1 and the spill ring heads to 0 itself:
    // cl_exec_kernel prologue -- no fill launch before every replay)
    ExecParams p = exec_params(begin, started_before);
    p.save_state = save_state ? 1 : 0;
    // replays of a planned program (build_plan): slot map, spill-free or split launches
    const bool planned = begin == 0 && trace_n == 0 && plan_ops == (int64_t)ops.size();
    if (planned) {
      p.inst_map = plan_map ? d_map.p : nullptr;
      p.nospill = plan_nospill ? 1 : 0;
      p.split_slot = plan_split;
    }
    // the first fresh full run of a program is the probe: per-instance spill flags (cleared
    // once per program, not per replay) and final ticks
    probe = begin == 0 && trace_n == 0 && !planned && plan_tried != (int64_t)ops.size();
    probe_ops = (int64_t)ops.size();
    probe_flags = probe && lay.ocap_log2 >= 0;
    if (probe_flags) {
      HIP_TRY(hipMemsetAsync(d_spill_inst.p, 0, (size_t)n_inst, stream));
      p.spill_flag = d_spill_inst.p;
    }
    if (p.split_slot > 0 && !stream2) {
      HIP_TRY(hipStreamCreateWithFlags(&stream2, hipStreamNonBlocking));
      HIP_TRY(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
      HIP_TRY(hipEventCreateWithFlags(&ev_join, hipEventDisableTiming));
    }
    if (ev_used == 256 && (rc = fold_events())) return rc;
    if (ev_used == ev_pool.size()) {
      LaunchEvents le;  // timing only: no cache writeback per record
      HIP_TRY(hipEventCreateWithFlags(&le.start, hipEventDisableSystemFence));
      HIP_TRY(hipEventCreateWithFlags(&le.stop, hipEventDisableSystemFence));
      HIP_TRY(hipEventCreateWithFlags(&le.stop2, hipEventDisableSystemFence));
      HIP_TRY(hipEventCreateWithFlags(&le.start2, hipEventDisableSystemFence));
      ev_pool.push_back(le);
    }
    ev_last = ev_used;
    auto& pr = ev_pool[ev_used++];
    pr.stop2_used = 0;
    // the dispatch records both events (the kernel's own start/end timestamps): two
    // hipEventRecord packets around it cost 0.7 us more per launch (C2 0.1816 -> 0.1809 ms per
    // step) and bracketed ~1 us of packet processing into the kernel time
    // split replays back to back do not join stream2 (r03 A/B: joining every replay measured slower)
    const bool pipe = planned && p.split_slot > 0 && p.split_slot < n_inst && stream2 && !save_state;
    if (!pipe && (rc = join_stream2())) return rc;
    // (a replay's stream2 half waits for `stream` only when `stream` got other work since the
    // last fork: consecutive replays touch disjoint instances on the two streams.  C3 per replay,
    // forking every replay / only then: 2^17 0.2391-0.2394 / 0.2370-0.2371 ms, 2^20
    // 1.6146-1.6151 / 1.6104-1.6113 ms, gpurun_out/r05z)
    const ExecLaunch el{stream, pr.start, pr.stop, stream2, ev_fork, ev_join, (!pipe || s_dirty) ? 1 : 0,
                        pipe ? 0 : 1, pr.stop2, &pr.stop2_used, pr.start2};
    // the instance-per-lane kernel, compiled for this topology, wherever it fits (N <= 16, every
    // degree <= 4) and the batch fills the chip with one instance per lane (AUTO); the
    // node-parallel kernel otherwise, or when run-time compilation failed
    const bool lanes = engine != CL_ENGINE_NODES && lanes_fit(p) &&
                       (engine == CL_ENGINE_LANES ||
                        ((int64_t)n_inst >= kLanesAutoMinInstances && std::max(max_out, max_in) >= 2));
    if (engine == CL_ENGINE_LANES && !lanes)
      return set_err(CL_E_LIMIT, "the instance-per-lane kernel needs <= %d nodes, degrees <= %d, <= 16 snapshots",
                     kLanesMaxNodes, kLanesMaxDegree);
    int e = lanes ? launch_lanes(p, d_topo.p, d_ops.p, d_sched.p, el) : launch_exec(p, d_topo.p, d_ops.p, d_sched.p, el);
    if (lanes && e == (int)hipErrorInvalidImage) {
      if (engine == CL_ENGINE_LANES)
        return set_err(CL_E_DEVICE, "instance-per-lane kernel compilation failed: %s", lanes_error());
      std::fprintf(stderr, "clsnap: instance-per-lane kernel unavailable, using the node-parallel kernel: %s\n",
                   lanes_error());
      engine = CL_ENGINE_NODES;
      e = launch_exec(p, d_topo.p, d_ops.p, d_sched.p, el);
    }
    last_engine = lanes && engine != CL_ENGINE_NODES ? CL_ENGINE_LANES : CL_ENGINE_NODES;
    if (pipe) {
      s2_live = true;
      s_dirty = false;
    }
    if (e != 0) return set_err(CL_E_DEVICE, "exec kernel launch failed: %s", hipGetErrorString((hipError_t)e));
    timed = true;
    executed = (int32_t)ops.size();
    need_fresh = false;
    state_valid = save_state;  // a rerun leaves no resumable image: the next flush replays
    h_valid = false;
    return CL_OK;
  }

  // The launcher's specialized kernels (and so split replays) serve this layout: unrolled
  // degree bound, staged delays, 2 / 4 / 8 LDS ring slots (cl_kernels.hip launch_exec_d).
  bool specialized() const {
    const int32_t d = std::max(std::max(max_out, max_in), 1);
    return degree_bound(d) <= kUnrollMaxD && lay.x_delay > 0 && lay.cap_log2 >= 1 && lay.cap_log2 <= 3;
  }

  int sync() {
    if (!dev_ready) return CL_OK;
    HIP_TRY(hipSetDevice(device));
    // a pipelined replay's stream2 half (s2_live) writes results too: `stream` waits for it
    // first, whichever path reached here (cl_wait_snapshot took the lock without
    // SIM_CHECK and could read snap_tick while the spill-capable half still ran)
    if (s2_live) {
      const int jrc = join_stream2();
      if (jrc) return jrc;
    }
    HIP_TRY(hipStreamSynchronize(stream));
    if (probe) {
      probe = false;
      int rc = build_plan();
      if (rc) return rc;
    }
    return CL_OK;
  }

  // Sum over waves of the longest instance (wave-ticks) of a slot order.
  int64_t wave_ticks(const std::vector<int32_t>& t, const std::vector<int32_t>& order, int64_t lo, int64_t hi) const {
    const int64_t ipw = std::max(lay.ipw, 1);
    int64_t sum = 0;
    for (int64_t w = lo; w < hi; w += ipw) {
      int32_t m = 0;
      for (int64_t k = w; k < std::min<int64_t>(w + ipw, hi); ++k) m = std::max(m, t[(size_t)order[(size_t)k]]);
      sum += m;
    }
    return sum;
  }

  // The replay plan from the probe's final ticks and spill flags (see d_spill_inst).
  int build_plan() {
    plan_tried = probe_ops;
    plan_map = plan_nospill = false;
    plan_split = plan_spilled = 0;
    // the length of an instance's replay: its final tick (one tick-loop iteration per tick)
    std::vector<int32_t> t((size_t)n_inst);
    HIP_TRY(hipMemcpy2D(t.data(), sizeof(int32_t), d_regs.p + R_TIME, R_NUM * sizeof(int32_t), sizeof(int32_t),
                        t.size(), hipMemcpyDeviceToHost));
    std::vector<uint8_t> sp((size_t)n_inst, 0);
    if (probe_flags) HIP_TRY(hipMemcpy(sp.data(), d_spill_inst.p, sp.size(), hipMemcpyDeviceToHost));
    std::vector<int32_t> clean, spilled, ident((size_t)n_inst);
    for (int64_t i = 0; i < n_inst; ++i) {
      ident[(size_t)i] = (int32_t)i;
      (sp[(size_t)i] ? spilled : clean).push_back((int32_t)i);
    }
    plan_spilled = (int64_t)spilled.size();
    plan_nospill = spilled.empty();
    // length order of the clean instances: one global counting sort by final tick (sorting
    // within windows of 64 waves instead, to keep each window's scattered per-instance stores
    // close in time, measured C3 2.71 -> 2.96 ms: the global order is kept)
    int32_t mx = 0;
    for (int32_t x : t) mx = std::max(mx, std::max(x, 0));
    std::vector<int64_t> start((size_t)mx + 2, 0);
    for (int32_t i : clean) start[(size_t)std::max(t[(size_t)i], 0) + 1]++;
    for (size_t k = 1; k < start.size(); ++k) start[k] += start[k - 1];
    std::vector<int32_t> by_len(clean.size());
    for (int32_t i : clean) by_len[(size_t)start[(size_t)std::max(t[(size_t)i], 0)]++] = i;
    // longest waves first (LPT): the dispatcher starts workgroups in slot order as resident
    // ones retire, so the last to start are the shortest and the grid drains evenly
    std::reverse(by_len.begin(), by_len.end());
    // worth it only when it removes enough wave-ticks to pay for the scattered stores (C3:
    // 43.9 -> 39.5 ticks per wave, kept; C2: 55.8 -> 52.8, measured slower mapped)
    const int64_t nc = (int64_t)clean.size();
    const int64_t ipw = std::max(lay.ipw, 1);
    // split replays: the clean instances' whole waves on the spill-free kernel (a wave that
    // holds a spilling instance runs spill-capable), when the launcher's kernels can split
    const bool split = !spilled.empty() && specialized();
    // a split launches through the map anyway (its scattered result stores are paid), so the
    // clean instances then go in length order too (C2: 0.1829 -> 0.1807 ms per step)
    const bool sort = n_inst >= kMapMinInstances &&
                      (split || wave_ticks(t, by_len, 0, nc) * 100 <= wave_ticks(t, clean, 0, nc) * kMapPct);
    std::vector<int32_t> order = sort ? by_len : clean;
    order.insert(order.end(), spilled.begin(), spilled.end());
    if (split) plan_split = nc / ipw * ipw;
    plan_map = sort || plan_split > 0;
    if (plan_map) {
      int rc = d_map.ensure(order.size());
      if (rc) return rc;
      HIP_TRY(hipMemcpy(d_map.p, order.data(), order.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    }
    plan_ops = probe_ops;
    return CL_OK;
  }

  int flush() {
    bool ran = false;
    if (!frozen || executed != (int32_t)ops.size() || need_fresh) {
      int rc = launch(false, true);
      if (rc) return rc;
      ran = true;
    }
    int rc = sync();
    if (rc == CL_OK && ran) {
      ++exec_gen;
      executed_cv.notify_all();
    }
    return rc;
  }

  // Instances of [lo, hi) in which snapshot sid has completed, as of every event issued
  // so far (pending events are executed; no tick is added), and how many of the others
  // are frozen (a FATAL / HANG / engine-limit status: their snapshot can never complete).
  int count_complete(int32_t sid, int64_t lo, int64_t hi, int64_t* n, int64_t* n_frozen = nullptr) {
    int rc = flush();
    if (rc) return rc;
    std::vector<int32_t> plane((size_t)std::max<int64_t>(hi - lo, 0)), stat(plane.size());
    if (h_valid) {
      for (int64_t i = lo; i < hi; ++i) {
        plane[(size_t)(i - lo)] = tick_at(sid, i);
        stat[(size_t)(i - lo)] = reg(i, R_STATUS);
      }
    } else if (hi > lo) {  // (instance-major rows: one strided copy each)
      HIP_TRY(hipMemcpy2D(plane.data(), sizeof(int32_t), d_snap_tick.p + (size_t)lo * s_cap + sid, s_cap * sizeof(int32_t),
                          sizeof(int32_t), plane.size(), hipMemcpyDeviceToHost));
      HIP_TRY(hipMemcpy2D(stat.data(), sizeof(int32_t), d_regs.p + (size_t)lo * R_NUM + R_STATUS, R_NUM * sizeof(int32_t),
                          sizeof(int32_t), stat.size(), hipMemcpyDeviceToHost));
    }
    const int32_t *t = plane.data(), *st = stat.data();
    int64_t c = 0, f = 0;
    for (int64_t i = 0; i < hi - lo; ++i) {
      c += t[i] >= 0;
      f += t[i] < 0 && st[i] != ST_OK;
    }
    *n = c;
    if (n_frozen) *n_frozen = f;
    return CL_OK;
  }

  int fetch() {
    int rc = flush();
    if (rc) return rc;
    if (h_valid) return CL_OK;
    if (!dev_ready) return set_err(CL_E_STATE, "nothing has run on the device yet");
    const int n = (int)ids.size();
    h_regs.resize((size_t)R_NUM * stride);
    h_snap_tick.resize((size_t)s_cap * stride);
    h_tok.resize((size_t)n * stride);
    HIP_TRY(hipMemcpy(h_regs.data(), d_regs.p, h_regs.size() * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(h_snap_tick.data(), d_snap_tick.p, h_snap_tick.size() * 4, hipMemcpyDeviceToHost));
    if (n) HIP_TRY(hipMemcpy(h_tok.data(), d_fin_tok.p, h_tok.size() * 4, hipMemcpyDeviceToHost));
    h_valid = true;
    return CL_OK;
  }

  int32_t reg(int64_t inst, int r) const { return h_regs[(size_t)inst * R_NUM + r]; }
  int32_t tick_at(int sid, int64_t inst) const { return h_snap_tick[(size_t)inst * s_cap + sid]; }
  // The node snapshot records of one (snapshot, instance): N * rw words (tokenMap entry of
  // node v at v * rw, the cursor word of channel c at ch_slot[c]).
  int records(int sid, int64_t inst, std::vector<uint32_t>* out) const {
    const size_t w = ids.size() * (size_t)lay.rw;
    out->resize(w);
    HIP_TRY(hipMemcpy(out->data(), d_snap_nod.p + ((size_t)sid * stride + inst) * w, w * 4, hipMemcpyDeviceToHost));
    return CL_OK;
  }

  SumParams sum_params() const {
    SumParams p{};
    p.n_nodes = (int32_t)ids.size();
    p.n_ch = (int32_t)ch_dst.size();
    p.s_cap = s_cap;
    p.n_sids = n_sids;
    p.n_inst = n_inst;
    p.stride = stride;
    p.regs = d_regs.p;
    p.rw = lay.rw;
    p.snap_nod = d_snap_nod.p;
    p.ch_slot = d_ch_slot.p;
    p.snap_tick = d_snap_tick.p;
    p.fin_tok = d_fin_tok.p;
    p.hist_off = d_hist.p;
    p.hist_val = d_hist.p + hist.size() + 1;
    p.total_tokens = total_tokens;
    return p;
  }

  // CollectSnapshot of instances [lo, hi) packed on the device (cl_pack_count / cl_pack_fill):
  // the packed arrays stay in d_pk_*; *total = messages.  Times the kernels (cl_collect_time).
  int pack(int32_t sid, int64_t lo, int64_t hi, int64_t* total) {
    int rc = flush();
    if (rc) return rc;
    if (!dev_ready) return set_err(CL_E_STATE, "nothing has run on the device yet");
    HIP_TRY(hipSetDevice(device));
    if ((rc = upload_hist())) return rc;
    const int64_t n = hi - lo;
    const int N = (int)ids.size(), C = (int)ch_dst.size();
    if ((rc = d_pk_tok.ensure((size_t)std::max<int64_t>(n, 1) * N)) || (rc = d_pk_done.ensure((size_t)n + 1)) ||
        (rc = d_pk_cnt.ensure((size_t)n + 1)) || (rc = d_pk_bsum.ensure((size_t)(n / kScanItems + 1))) ||
        (rc = d_pk_off.ensure((size_t)n * C + 1)))
      return rc;
    for (auto& e : pk_ev)
      if (!e) HIP_TRY(hipEventCreate(&e));
    PackParams p{};
    p.n_nodes = N;
    p.n_ch = C;
    p.s_cap = s_cap;
    p.rw = lay.rw;
    p.sid = sid;
    p.lo = lo;
    p.n = n;
    p.stride = stride;
    p.snap_nod = d_snap_nod.p;
    p.snap_tick = d_snap_tick.p;
    p.ch_slot = d_ch_slot.p;
    p.hist_off = d_hist.p;
    p.hist_val = d_hist.p + hist.size() + 1;
    p.tokens = d_pk_tok.p;
    p.complete = d_pk_done.p;
    p.count = d_pk_cnt.p;
    p.bsum = d_pk_bsum.p;
    p.offsets = d_pk_off.p;
    HIP_TRY(hipEventRecord(pk_ev[0], stream));
    int e = launch_pack_count(p, stream);
    if (e) return set_err(CL_E_DEVICE, "pack kernels: %s", hipGetErrorString((hipError_t)e));
    long long tot = 0;
    HIP_TRY(hipMemcpyAsync(&tot, d_pk_cnt.p + n, sizeof tot, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    if ((rc = d_pk_msg.ensure((size_t)std::max<long long>(tot, 1)))) return rc;
    p.msgs = d_pk_msg.p;
    e = launch_pack_fill(p, stream);
    if (e) return set_err(CL_E_DEVICE, "pack kernels: %s", hipGetErrorString((hipError_t)e));
    HIP_TRY(hipEventRecord(pk_ev[1], stream));
    pk_timed = true;
    *total = tot;
    return CL_OK;
  }

  int append(Op op) {
    int rc = freeze();
    if (rc) return rc;
    ops.push_back(op);
    return CL_OK;
  }
};

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

const char* cl_last_error(void) { return last_error(); }

const char* cl_status_string(int32_t code) {
  switch (code) {
    case CL_INST_OK: return "ok";
    case CL_INST_FATAL_INSUFFICIENT_TOKENS: return "fatal: insufficient tokens (node.go:113-116)";
    case CL_INST_FATAL_UNKNOWN_DEST: return "fatal: unknown dest (node.go:121-124)";
    case CL_INST_FIFO_OVERFLOW: return "fifo overflow (engine limit)";
    case CL_INST_HANG: return "hang: snapshot never completed";
    case CL_INST_DELAY_EXHAUSTED: return "delay schedule exhausted";
    case CL_INST_HIST_OVERFLOW: return "token history overflow (engine limit)";
    default: return "unknown";
  }
}

// Every ABI call but cl_rerun first joins a pipelined replay's stream2 half (cl_sim::s2_live).
#define SIM_CHECK_NOJOIN(s)                                         \
  if (!(s)) return set_err(CL_E_INVALID, "null cl_sim handle");  \
  std::lock_guard<std::recursive_mutex> sim_lock_((s)->mu)
#define SIM_CHECK(s)                                                \
  SIM_CHECK_NOJOIN(s);                                              \
  if ((s)->s2_live) {                                               \
    const int jrc_ = const_cast<cl_sim*>(s)->join_stream2();        \
    if (jrc_) return jrc_;                                          \
  }

int cl_sim_create(int64_t n_instances, cl_sim** out) {
  if (!out || n_instances <= 0) return set_err(CL_E_INVALID, "n_instances must be > 0");
  cl_sim* s = new cl_sim();
  s->n_inst = n_instances;
  s->stride = (n_instances + kWave - 1) / kWave * kWave;
  *out = s;
  return CL_OK;
}

int cl_sim_destroy(cl_sim* sim) {
  if (sim) {
    // wake every thread blocked in cl_wait_snapshot and wait until it has left; no other
    // call may be in flight or start on this sim once destroy is called
    std::unique_lock<std::recursive_mutex> lk(sim->mu);
    sim->closing = true;
    ++sim->exec_gen;
    sim->executed_cv.notify_all();
    sim->executed_cv.wait(lk, [&] { return sim->waiters == 0; });
  }
  delete sim;
  return CL_OK;
}

int cl_add_node(cl_sim* sim, const char* id, int64_t tokens) {
  SIM_CHECK(sim);
  if (!id) return set_err(CL_E_INVALID, "null id");
  if (sim->frozen) return set_err(CL_E_STATE, "AddNode after events started is not supported");
  if (sim->node_of(id) >= 0) return set_err(CL_E_DUPLICATE_NODE, "node %s already exists", id);
  if (tokens < INT32_MIN || tokens > INT32_MAX) return set_err(CL_E_LIMIT, "token count out of int32 range");
  sim->id_index[id] = (int)sim->ids.size();
  sim->ids.emplace_back(id);
  sim->init_tokens.push_back(tokens);
  int64_t total = 0;
  for (auto t : sim->init_tokens) total += t;
  if (total > INT32_MAX || total < INT32_MIN) return set_err(CL_E_LIMIT, "total tokens out of int32 range");
  return CL_OK;
}

int cl_add_link(cl_sim* sim, const char* src, const char* dest) {
  SIM_CHECK(sim);
  const int a = sim->node_of(src), b = sim->node_of(dest);
  if (a < 0) return set_err(CL_E_UNKNOWN_NODE, "Node %s does not exist", src ? src : "(null)");
  if (b < 0) return set_err(CL_E_UNKNOWN_NODE, "Node %s does not exist", dest ? dest : "(null)");
  if (sim->frozen) return set_err(CL_E_STATE, "AddLink after events started is not supported");
  if (a == b) return CL_OK;  // node.go:88-90
  for (auto& l : sim->links)
    if (l.first == a && l.second == b) return CL_OK;  // replacement of an empty queue
  sim->links.emplace_back(a, b);
  return CL_OK;
}

int cl_read_topology_text(cl_sim* sim, const char* text) {
  SIM_CHECK(sim);
  if (!text) return set_err(CL_E_INVALID, "null text");
  int64_t left = -1;
  for (const std::string& line : go_lines(text)) {
    if (!line.empty() && line[0] == '#') continue;
    if (left < 0) {
      if (!go_atoi(line, &left)) return set_err(CL_E_PARSE, "bad node count line: %s", line.c_str());
      continue;
    }
    auto f = go_fields(line);
    if (f.size() != 2) return set_err(CL_E_PARSE, "Expected 2 tokens in line: %s", line.c_str());
    int rc;
    if (left > 0) {
      int64_t tok;
      if (!go_atoi(f[1], &tok)) return set_err(CL_E_PARSE, "bad token count: %s", f[1].c_str());
      if ((rc = cl_add_node(sim, f[0].c_str(), tok))) return rc;
      left--;
    } else if ((rc = cl_add_link(sim, f[0].c_str(), f[1].c_str()))) {
      return rc;
    }
  }
  return CL_OK;
}

int cl_read_topology_file(cl_sim* sim, const char* path) {
  SIM_CHECK(sim);
  std::string text;
  if (!path || !read_file(path, &text)) return set_err(CL_E_IO, "cannot read %s", path ? path : "(null)");
  return cl_read_topology_text(sim, text.c_str());
}

int cl_set_device(cl_sim* sim, int32_t device_ordinal) {
  SIM_CHECK(sim);
  if (sim->dev_ready) return set_err(CL_E_STATE, "device already selected");
  sim->device = device_ordinal;
  return CL_OK;
}

int cl_set_limits(cl_sim* sim, int32_t fifo_lds_slots, int64_t max_drain_ticks) {
  SIM_CHECK(sim);
  if (max_drain_ticks < 0) return set_err(CL_E_INVALID, "max_drain_ticks must be >= 0");
  sim->max_drain = max_drain_ticks;
  if (fifo_lds_slots == 0) {  // automatic
    if (!sim->auto_cap) sim->need_fresh = true;
    sim->auto_cap = true;
    return CL_OK;
  }
  int l = 0;
  while ((1 << l) < fifo_lds_slots) ++l;
  if (fifo_lds_slots < 2 || fifo_lds_slots > 64 || (1 << l) != fifo_lds_slots)
    return set_err(CL_E_INVALID, "fifo_lds_slots must be 0 (automatic) or a power of two in [2, 64]");
  if (l != sim->cap_log2 || sim->auto_cap) sim->need_fresh = true;
  sim->cap_log2 = l;
  sim->auto_cap = false;
  return CL_OK;
}

int cl_set_delay_go_seeds(cl_sim* sim, int64_t seed_base) {
  SIM_CHECK(sim);
  sim->plan_ops = sim->plan_tried = -1;
  sim->go_seeds = true;
  sim->seed_base = seed_base;
  sim->dev_draws = -1;
  sim->need_fresh = true;
  return CL_OK;
}

int cl_set_delay_schedule(cl_sim* sim, const uint8_t* delays, int64_t draws_per_instance) {
  SIM_CHECK(sim);
  sim->plan_ops = sim->plan_tried = -1;
  if (!delays || draws_per_instance <= 0) return set_err(CL_E_INVALID, "empty schedule");
  const size_t n = (size_t)(draws_per_instance * sim->n_inst);
  for (size_t i = 0; i < n; ++i)
    if (delays[i] >= 5) return set_err(CL_E_INVALID, "delay %u at %zu outside [0, maxDelay)", delays[i], i);
  sim->user_sched.assign(delays, delays + n);
  sim->user_draws = draws_per_instance;
  sim->go_seeds = false;
  sim->dev_draws = -1;
  sim->need_fresh = true;
  return CL_OK;
}

int cl_send_tokens(cl_sim* sim, const char* src, const char* dest, int64_t n) {
  SIM_CHECK(sim);
  int rc = sim->freeze();
  if (rc) return rc;
  const int a = sim->node_of(src);
  if (a < 0) return set_err(CL_E_UNKNOWN_NODE, "send from unknown node %s", src ? src : "(null)");
  if (n < 0 || n > kMaxPayload) return set_err(CL_E_LIMIT, "token count %lld outside [0, %d]", (long long)n, kMaxPayload);
  const int b = sim->node_of(dest);
  const int ra = sim->rank_of[a];
  const int c = b < 0 ? -1 : sim->channel_of(ra, sim->rank_of[b]);
  const int ko = c < 0 ? -1 : c - sim->out_off[ra];  // out-index of the link at its sender
  if (c >= 0) {
    if ((int64_t)sim->hist[c].size() >= kMaxChannelTokens)
      return set_err(CL_E_LIMIT, "more than %d token messages on one channel", kMaxChannelTokens);
    sim->hist[c].push_back((int32_t)n);
    sim->depth_bound[c]++;
  }
  sim->sends++;
  return sim->append(Op{OP_SEND, ra, ko, (int32_t)n});
}

int cl_start_snapshot(cl_sim* sim, const char* node, int32_t* out_sid) {
  SIM_CHECK(sim);
  int rc = sim->freeze();
  if (rc) return rc;
  const int a = sim->node_of(node);
  if (a < 0) return set_err(CL_E_UNKNOWN_NODE, "snapshot at unknown node %s", node ? node : "(null)");
  if (sim->n_sids >= kMaxSnapshots) return set_err(CL_E_LIMIT, "more than %d snapshots", kMaxSnapshots);
  const int32_t sid = sim->n_sids++;
  for (auto& d : sim->depth_bound) d++;
  if (out_sid) *out_sid = sid;
  const int r = sim->rank_of[a];
  return sim->append(Op{OP_SNAP, r, sid, sim->out_off[r + 1] - sim->out_off[r]});
}

int cl_tick(cl_sim* sim, int32_t n) {
  SIM_CHECK(sim);
  int rc = sim->freeze();
  if (rc) return rc;
  if (n <= 0) return CL_OK;  // for i := 0; i < numTicks; ... (test_common.go:115)
  if (sim->time_bound + n > kMaxTime)
    return set_err(CL_E_LIMIT, "simulated time would exceed %d ticks", kMaxTime);
  sim->time_bound += n;
  if (!sim->ops.empty() && sim->ops.back().kind == OP_TICK && sim->executed < (int32_t)sim->ops.size()) {
    sim->ops.back().a += n;  // merge consecutive ticks of one pending run
  } else if ((rc = sim->append(Op{OP_TICK, n, 0, 0}))) {
    return rc;
  }
  sim->notify_waiters();
  return CL_OK;
}

int cl_drain(cl_sim* sim) {
  SIM_CHECK(sim);
  int rc = sim->freeze();
  if (rc) return rc;
  const int64_t extra = 6;  // maxDelay + 1 (test_common.go:135-137)
  int64_t room = kMaxTime - sim->time_bound - extra;
  if (room < 0) return set_err(CL_E_LIMIT, "simulated time would exceed %d ticks", kMaxTime);
  const int64_t cap = std::min(sim->max_drain, room);
  sim->time_bound += cap + extra;
  if ((rc = sim->append(Op{OP_DRAIN, (int32_t)cap, (int32_t)extra, 0}))) return rc;
  sim->notify_waiters();
  return CL_OK;
}

int cl_read_events_text(cl_sim* sim, const char* text, int32_t* n_snapshots) {
  SIM_CHECK(sim);
  if (!text) return set_err(CL_E_INVALID, "null text");
  int32_t snaps = 0;
  for (const std::string& line : go_lines(text)) {
    if (line == "#") continue;  // strings.HasPrefix("#", line) (test_common.go:90, sic)
    auto f = go_fields(line);
    if (f.empty()) return set_err(CL_E_PARSE, "empty event line");
    int rc;
    if (f[0] == "send") {
      int64_t n;
      if (f.size() < 4 || !go_atoi(f[3], &n)) return set_err(CL_E_PARSE, "bad send line: %s", line.c_str());
      rc = cl_send_tokens(sim, f[1].c_str(), f[2].c_str(), n);
    } else if (f[0] == "snapshot") {
      if (f.size() < 2) return set_err(CL_E_PARSE, "bad snapshot line: %s", line.c_str());
      snaps++;
      rc = cl_start_snapshot(sim, f[1].c_str(), nullptr);
    } else if (f[0] == "tick") {
      int64_t n = 1;
      if (f.size() > 1 && !go_atoi(f[1], &n)) return set_err(CL_E_PARSE, "bad tick line: %s", line.c_str());
      if (n > INT32_MAX) return set_err(CL_E_LIMIT, "tick count too large");
      rc = cl_tick(sim, (int32_t)std::max<int64_t>(n, 0));
    } else {
      return set_err(CL_E_PARSE, "Unknown event command: %s", f[0].c_str());
    }
    if (rc) return rc;
  }
  if (n_snapshots) *n_snapshots = snaps;
  return cl_drain(sim);
}

int cl_read_events_file(cl_sim* sim, const char* path, int32_t* n_snapshots) {
  SIM_CHECK(sim);
  std::string text;
  if (!path || !read_file(path, &text)) return set_err(CL_E_IO, "cannot read %s", path ? path : "(null)");
  return cl_read_events_text(sim, text.c_str(), n_snapshots);
}

int cl_flush(cl_sim* sim) {
  SIM_CHECK(sim);
  return sim->flush();
}

int cl_rerun(cl_sim* sim) {
  SIM_CHECK_NOJOIN(sim);
  const int rc = sim->launch(true, false);
  if (rc == CL_OK) sim->notify_waiters();  // a blocked collector re-checks against the new run
  return rc;
}

int cl_replay_spill_free(cl_sim* sim, int32_t* on) {
  SIM_CHECK(sim);
  if (!on) return set_err(CL_E_INVALID, "null output");
  int rc = sim->sync();
  if (rc) return rc;
  *on = sim->lay.ocap_log2 < 0 || (sim->plan_ops == (int64_t)sim->ops.size() && sim->plan_nospill) ? 1 : 0;
  return CL_OK;
}

int cl_replay_split(cl_sim* sim, int64_t* spill_instances, int64_t* split_slot) {
  SIM_CHECK(sim);
  if (!spill_instances || !split_slot) return set_err(CL_E_INVALID, "null output");
  int rc = sim->sync();  // (a pending probe is evaluated here)
  if (rc) return rc;
  const bool planned = sim->plan_ops == (int64_t)sim->ops.size();
  *spill_instances = planned ? sim->plan_spilled : -1;
  *split_slot = planned ? sim->plan_split : 0;
  return CL_OK;
}

int cl_replay_mapped(cl_sim* sim, int32_t* on) {
  SIM_CHECK(sim);
  if (!on) return set_err(CL_E_INVALID, "null output");
  int rc = sim->sync();  // (a pending map probe is evaluated here)
  if (rc) return rc;
  *on = sim->plan_ops == (int64_t)sim->ops.size() && sim->plan_map ? 1 : 0;
  return CL_OK;
}

int cl_synchronize(cl_sim* sim) {
  SIM_CHECK(sim);
  return sim->sync();
}

int cl_set_exec_engine(cl_sim* sim, int32_t engine) {
  SIM_CHECK(sim);
  if (engine != CL_ENGINE_AUTO && engine != CL_ENGINE_NODES && engine != CL_ENGINE_LANES)
    return set_err(CL_E_INVALID, "unknown exec engine %d", engine);
  if (engine != sim->engine) {
    // the next launch replays the program from the start on the chosen kernel (results are the
    // same; the resumable state image is shared by both kernels)
    sim->engine = engine;
    sim->plan_ops = sim->plan_tried = -1;
  }
  return CL_OK;
}

int cl_exec_engine(cl_sim* sim, int32_t* engine) {
  SIM_CHECK(sim);
  if (!engine) return set_err(CL_E_INVALID, "null output");
  *engine = sim->last_engine;
  return CL_OK;
}

int cl_lanes_compile_check(cl_sim* sim, double* compile_ms, char* log, int64_t log_cap) {
  SIM_CHECK(sim);
  int rc = sim->freeze();
  if (rc) return rc;
  if (sim->ids.empty()) return set_err(CL_E_STATE, "the topology has no nodes");
  ExecParams p{};
  int64_t row = 0;
  p.lay = sim->plan_layout(nullptr, nullptr, &row);
  p.n_nodes = (int32_t)sim->ids.size();
  p.n_ch = (int32_t)sim->ch_dst.size();
  p.sched_row = row;
  p.lt = sim->lanes_topo();
  if (!lanes_fit(p)) return set_err(CL_E_LIMIT, "the topology does not fit the instance-per-lane kernel");
  std::string l;
  rc = lanes_compile_only(p, compile_ms, &l);
  if (log && log_cap > 0) {
    const size_t n = std::min<size_t>(l.size(), (size_t)log_cap - 1);
    std::memcpy(log, l.data(), n);
    log[n] = 0;
  }
  return rc ? set_err(CL_E_DEVICE, "instance-per-lane kernel compilation failed") : CL_OK;
}

int cl_jit_stats(double* compile_ms, int64_t* compiles) {
  clsnap::lanes_jit_stats(compile_ms, compiles);
  return CL_OK;
}

int cl_debug_poison_outputs(cl_sim* sim) {
  SIM_CHECK(sim);
  if (!sim->dev_ready || !sim->d_regs.p) return CL_OK;
  HIP_TRY(hipSetDevice(sim->device));
  const int n = (int)sim->ids.size();
  const size_t nod = (size_t)sim->s_cap * n * sim->lay.rw * sim->stride;
  HIP_TRY(hipMemsetAsync(sim->d_snap_nod.p, 0xA5, nod * sizeof(uint32_t), sim->stream));
  HIP_TRY(hipMemsetAsync(sim->d_snap_tick.p, 0xA5, (size_t)sim->s_cap * sim->stride * sizeof(int32_t), sim->stream));
  HIP_TRY(hipMemsetAsync(sim->d_regs.p, 0xA5, (size_t)R_NUM * sim->stride * sizeof(int32_t), sim->stream));
  HIP_TRY(hipMemsetAsync(sim->d_fin_tok.p, 0xA5, (size_t)n * sim->stride * sizeof(int32_t), sim->stream));
  sim->h_valid = false;
  return CL_OK;
}

int cl_last_kernel_ms(cl_sim* sim, double* ms) {
  SIM_CHECK(sim);
  if (!ms) return set_err(CL_E_INVALID, "null output");
  if (!sim->timed) return set_err(CL_E_STATE, "no kernel has run");
  int rc = sim->sync();
  if (rc) return rc;
  float f = 0.f;
  if ((rc = sim->launch_ms(sim->ev_pool[sim->ev_last], &f))) return rc;
  *ms = f;
  return CL_OK;
}

int cl_kernel_time(cl_sim* sim, double* total_ms, int64_t* launches) {
  SIM_CHECK(sim);
  if (!total_ms || !launches) return set_err(CL_E_INVALID, "null output");
  int rc = sim->sync();
  if (rc) return rc;
  if (sim->dev_ready && (rc = sim->fold_events())) return rc;
  *total_ms = sim->ev_folded_ms;
  *launches = sim->ev_folded_n;
  sim->ev_folded_ms = 0;
  sim->ev_folded_n = 0;
  return CL_OK;
}

int cl_num_nodes(const cl_sim* sim, int32_t* n) {
  SIM_CHECK(sim);
  *n = (int32_t)sim->ids.size();
  return CL_OK;
}

int cl_node_id(const cl_sim* sim, int32_t rank, const char** id) {
  SIM_CHECK(sim);
  if (!sim->frozen) {
    int rc = const_cast<cl_sim*>(sim)->freeze();
    if (rc) return rc;
  }
  if (rank < 0 || rank >= (int32_t)sim->ids.size()) return set_err(CL_E_INVALID, "rank out of range");
  *id = sim->ids[sim->by_rank[rank]].c_str();
  return CL_OK;
}

int cl_num_channels(const cl_sim* sim, int32_t* n) {
  SIM_CHECK(sim);
  *n = (int32_t)sim->links.size();
  return CL_OK;
}

int cl_channel(const cl_sim* sim, int32_t ch, int32_t* src_rank, int32_t* dest_rank) {
  SIM_CHECK(sim);
  if (!sim->frozen) {
    int rc = const_cast<cl_sim*>(sim)->freeze();
    if (rc) return rc;
  }
  if (ch < 0 || ch >= (int32_t)sim->ch_dst.size()) return set_err(CL_E_INVALID, "channel out of range");
  *src_rank = sim->ch_src[ch];
  *dest_rank = sim->ch_dst[ch];
  return CL_OK;
}

int cl_num_snapshots(const cl_sim* sim, int32_t* n) {
  SIM_CHECK(sim);
  *n = sim->n_sids;
  return CL_OK;
}

int cl_num_instances(const cl_sim* sim, int64_t* n) {
  SIM_CHECK(sim);
  *n = sim->n_inst;
  return CL_OK;
}

int cl_delay_draws_needed(const cl_sim* sim, int64_t* draws) {
  SIM_CHECK(sim);
  *draws = sim->draws_needed();
  return CL_OK;
}

int cl_device_bytes(const cl_sim* sim, int64_t* bytes) {
  SIM_CHECK(sim);
  int64_t b = 0;
  b += sim->d_ops.n * sizeof(Op) + sim->d_topo.n * 4 + sim->d_sched.n + sim->d_state.n * 4 + sim->d_regs.n * 4;
  b += sim->d_snap_nod.n * 4 + sim->d_snap_tick.n * 4 + sim->d_ovf.n * 4;
  b += sim->d_ovh.n * 4 + sim->d_hist.n * 4 + sim->d_sums.n * 8 + sim->d_fin_tok.n * 4;
  *bytes = b;
  return CL_OK;
}

int cl_get_status(cl_sim* sim, int32_t* out) {
  SIM_CHECK(sim);
  int rc = sim->fetch();
  if (rc) return rc;
  for (int64_t i = 0; i < sim->n_inst; ++i) out[i] = sim->reg(i, R_STATUS);
  return CL_OK;
}

int cl_get_time(cl_sim* sim, int32_t* out) {
  SIM_CHECK(sim);
  int rc = sim->fetch();
  if (rc) return rc;
  for (int64_t i = 0; i < sim->n_inst; ++i) out[i] = sim->reg(i, R_TIME);
  return CL_OK;
}

int cl_node_tokens(cl_sim* sim, int64_t inst, int64_t* out) {
  SIM_CHECK(sim);
  if (inst < 0 || inst >= sim->n_inst) return set_err(CL_E_INVALID, "instance out of range");
  int rc = sim->fetch();
  if (rc) return rc;
  const size_t n = sim->ids.size();
  for (size_t r = 0; r < n; ++r) out[r] = sim->h_tok[(size_t)inst * n + r];
  return CL_OK;
}

int cl_snapshot_tick(cl_sim* sim, int32_t sid, int64_t inst, int32_t* tick) {
  SIM_CHECK(sim);
  if (inst < 0 || inst >= sim->n_inst || sid < 0 || sid >= sim->n_sids)
    return set_err(CL_E_INVALID, "snapshot/instance out of range");
  int rc = sim->fetch();
  if (rc) return rc;
  *tick = sim->tick_at(sid, inst);
  return CL_OK;
}

int cl_collect_snapshot(cl_sim* sim, int32_t sid, int64_t inst, int64_t* tokens, int64_t* msg_offsets,
                        int64_t* msg_tokens, int64_t msg_cap) {
  SIM_CHECK(sim);
  if (inst < 0 || inst >= sim->n_inst || sid < 0 || sid >= sim->n_sids)
    return set_err(CL_E_INVALID, "snapshot/instance out of range");
  int rc = sim->fetch();
  if (rc) return rc;
  if (sim->tick_at(sid, inst) < 0)
    return set_err(CL_E_NOT_COMPLETE, "snapshot %d has not completed in instance %lld", sid, (long long)inst);
  const int n = (int)sim->ids.size(), C = (int)sim->ch_dst.size();
  std::vector<uint32_t> rb;
  if ((rc = sim->records(sid, inst, &rb))) return rc;
  for (int v = 0; v < n; ++v) tokens[v] = (int32_t)rb[(size_t)v * sim->lay.rw];
  int64_t m = 0;
  bool fits = true;
  for (int c = 0; c < C; ++c) {
    msg_offsets[c] = m;
    const uint32_t rec = rb[sim->ch_slot[c]];
    const uint32_t b = rec & 0xffffu, e = rec >> 16;
    for (uint32_t k = b; k < e; ++k, ++m) {
      if (m < msg_cap) msg_tokens[m] = sim->hist[c][k];
      else fits = false;
    }
  }
  msg_offsets[C] = m;
  return fits ? CL_OK : set_err(CL_E_LIMIT, "msg_cap %lld < %lld messages", (long long)msg_cap, (long long)m);
}

int cl_poll_snapshot(cl_sim* sim, int32_t sid, int64_t inst_lo, int64_t inst_hi, int64_t* n_complete) {
  SIM_CHECK(sim);
  if (!n_complete) return set_err(CL_E_INVALID, "null output");
  if (sid < 0 || sid >= sim->n_sids || inst_lo < 0 || inst_hi > sim->n_inst || inst_lo > inst_hi)
    return set_err(CL_E_INVALID, "snapshot/instance range out of range");
  return sim->count_complete(sid, inst_lo, inst_hi, n_complete);
}

int cl_wait_snapshot(cl_sim* sim, int32_t sid, int64_t inst_lo, int64_t inst_hi, int64_t timeout_ms,
                     int64_t* n_complete) {
  if (!sim) return set_err(CL_E_INVALID, "null cl_sim handle");
  std::unique_lock<std::recursive_mutex> lk(sim->mu);
  if (sid < 0 || sid >= sim->n_sids || inst_lo < 0 || inst_hi > sim->n_inst || inst_lo > inst_hi)
    return set_err(CL_E_INVALID, "snapshot/instance range out of range");
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms < 0 ? 0 : timeout_ms);
  struct Waiting {  // registered while blocked, so cl_sim_destroy can wait for this thread
    cl_sim* s;
    explicit Waiting(cl_sim* x) : s(x) { ++s->waiters; }
    ~Waiting() {
      if (--s->waiters == 0 && s->closing) s->executed_cv.notify_all();
    }
  } waiting(sim);
  for (;;) {
    if (sim->closing) return set_err(CL_E_STATE, "the sim is being destroyed");
    // (the driver thread may have issued a pipelined replay since the last wake-up)
    if (sim->s2_live) {
      const int jrc = sim->join_stream2();
      if (jrc) return jrc;
    }
    int64_t n = 0, frozen = 0;
    int rc = sim->count_complete(sid, inst_lo, inst_hi, &n, &frozen);
    if (rc) return rc;
    if (n_complete) *n_complete = n;
    if (n == inst_hi - inst_lo) return CL_OK;
    if (n + frozen == inst_hi - inst_lo)  // the rest stopped at a fatal: they never complete
      return set_err(CL_E_NOT_COMPLETE, "snapshot %d: %lld of %lld instances complete, %lld stopped (status != ok)",
                     sid, (long long)n, (long long)(inst_hi - inst_lo), (long long)frozen);
    const uint64_t gen = sim->exec_gen;
    auto more = [&] { return sim->exec_gen != gen; };
    if (timeout_ms < 0) {
      sim->executed_cv.wait(lk, more);
    } else if (!sim->executed_cv.wait_until(lk, deadline, more)) {
      return set_err(CL_E_NOT_COMPLETE, "snapshot %d: %lld of %lld instances complete at the timeout", sid,
                     (long long)n, (long long)(inst_hi - inst_lo));
    }
  }
}

int cl_collect_snapshot_range(cl_sim* sim, int32_t sid, int64_t inst_lo, int64_t inst_hi, int64_t* tokens,
                              int32_t* complete, int64_t* msg_offsets, int64_t* msg_tokens, int64_t msg_cap) {
  SIM_CHECK(sim);
  if (sid < 0 || sid >= sim->n_sids || inst_lo < 0 || inst_hi > sim->n_inst || inst_lo > inst_hi)
    return set_err(CL_E_INVALID, "snapshot/instance range out of range");
  int64_t tot = 0;
  int rc = sim->pack(sid, inst_lo, inst_hi, &tot);
  if (rc) return rc;
  const int64_t n = inst_hi - inst_lo;
  const int N = (int)sim->ids.size(), C = (int)sim->ch_dst.size();
  if (complete) HIP_TRY(hipMemcpy(complete, sim->d_pk_done.p, (size_t)n * 4, hipMemcpyDeviceToHost));
  if (msg_offsets) HIP_TRY(hipMemcpy(msg_offsets, sim->d_pk_off.p, ((size_t)n * C + 1) * 8, hipMemcpyDeviceToHost));
  if (tokens) {  // (the int64 ABI widens on the host)
    std::vector<int32_t> t((size_t)n * N);
    if (!t.empty()) HIP_TRY(hipMemcpy(t.data(), sim->d_pk_tok.p, t.size() * 4, hipMemcpyDeviceToHost));
    for (size_t k = 0; k < t.size(); ++k) tokens[k] = t[k];
  }
  if (tot > msg_cap || (tot > 0 && !msg_tokens))
    return set_err(CL_E_LIMIT, "msg_cap %lld < %lld messages", (long long)msg_cap, (long long)tot);
  if (tot > 0) {
    std::vector<int32_t> m((size_t)tot);
    HIP_TRY(hipMemcpy(m.data(), sim->d_pk_msg.p, m.size() * 4, hipMemcpyDeviceToHost));
    for (size_t k = 0; k < m.size(); ++k) msg_tokens[k] = m[k];
  }
  return CL_OK;
}

int cl_collect_snapshot_packed(cl_sim* sim, int32_t sid, int64_t inst_lo, int64_t inst_hi, int32_t* tokens,
                               int32_t* complete, int64_t* msg_offsets, int32_t* msg_tokens, int64_t msg_cap,
                               int64_t* n_msgs) {
  SIM_CHECK(sim);
  if (sid < 0 || sid >= sim->n_sids || inst_lo < 0 || inst_hi > sim->n_inst || inst_lo > inst_hi)
    return set_err(CL_E_INVALID, "snapshot/instance range out of range");
  int64_t tot = 0;
  int rc = sim->pack(sid, inst_lo, inst_hi, &tot);
  if (rc) return rc;
  if (n_msgs) *n_msgs = tot;
  const size_t n = (size_t)(inst_hi - inst_lo), N = sim->ids.size(), C = sim->ch_dst.size();
  if (tokens && n) HIP_TRY(hipMemcpyAsync(tokens, sim->d_pk_tok.p, n * N * 4, hipMemcpyDeviceToHost, sim->stream));
  if (complete && n) HIP_TRY(hipMemcpyAsync(complete, sim->d_pk_done.p, n * 4, hipMemcpyDeviceToHost, sim->stream));
  if (msg_offsets) HIP_TRY(hipMemcpyAsync(msg_offsets, sim->d_pk_off.p, (n * C + 1) * 8, hipMemcpyDeviceToHost, sim->stream));
  const bool fits = tot <= msg_cap && (tot == 0 || msg_tokens);
  if (fits && tot > 0)
    HIP_TRY(hipMemcpyAsync(msg_tokens, sim->d_pk_msg.p, (size_t)tot * 4, hipMemcpyDeviceToHost, sim->stream));
  HIP_TRY(hipStreamSynchronize(sim->stream));
  return fits ? CL_OK : set_err(CL_E_LIMIT, "msg_cap %lld < %lld messages", (long long)msg_cap, (long long)tot);
}

int cl_collect_time(cl_sim* sim, double* device_ms) {
  SIM_CHECK(sim);
  if (!device_ms) return set_err(CL_E_INVALID, "null output");
  if (!sim->pk_timed) return set_err(CL_E_STATE, "no packed collect has run");
  HIP_TRY(hipStreamSynchronize(sim->stream));
  float f = 0.f;
  HIP_TRY(hipEventElapsedTime(&f, sim->pk_ev[0], sim->pk_ev[1]));
  *device_ms = f;
  return CL_OK;
}

int cl_get_counters(cl_sim* sim, int32_t only_ok, int64_t* out) {
  SIM_CHECK(sim);
  int rc = sim->fetch();
  if (rc) return rc;
  for (int k = 0; k < CL_NUM_COUNTERS; ++k) out[k] = 0;
  for (int64_t i = 0; i < sim->n_inst; ++i) {
    if (only_ok && sim->reg(i, R_STATUS) != ST_OK) continue;
    out[CL_CNT_PUSH] += (uint32_t)sim->reg(i, R_PUSH);
    out[CL_CNT_PEEK] += (uint32_t)sim->reg(i, R_PEEK);
    out[CL_CNT_POP_TOKEN] += (uint32_t)sim->reg(i, R_POP_TOK);
    out[CL_CNT_POP_MARKER] += (uint32_t)sim->reg(i, R_POP_MK);
    out[CL_CNT_COMPLETED] += sim->reg(i, R_NDONE);
    out[CL_CNT_INSTANCES] += 1;
    out[CL_CNT_TICKS] += sim->reg(i, R_TIME);
  }
  // recorded copies over completed snapshots: summed on the device from the node records
  HIP_TRY(hipSetDevice(sim->device));
  if ((rc = sim->d_rec2.ensure(2))) return rc;
  HIP_TRY(hipMemsetAsync(sim->d_rec2.p, 0, 2 * sizeof(unsigned long long), sim->stream));
  SumParams p = sim->sum_params();
  p.out = sim->d_rec2.p;
  int e = launch_recorded(p, sim->stream);
  if (e) return set_err(CL_E_DEVICE, "recorded-count kernel: %s", hipGetErrorString((hipError_t)e));
  unsigned long long r[2];
  HIP_TRY(hipMemcpyAsync(r, sim->d_rec2.p, sizeof r, hipMemcpyDeviceToHost, sim->stream));
  HIP_TRY(hipStreamSynchronize(sim->stream));
  out[CL_CNT_RECORDED] = (int64_t)r[only_ok ? 1 : 0];
  return CL_OK;
}

int cl_get_checksums(cl_sim* sim, int64_t* out) {
  SIM_CHECK(sim);
  int rc = sim->flush();
  if (rc) return rc;
  if (!sim->dev_ready) return set_err(CL_E_STATE, "nothing has run on the device yet");
  HIP_TRY(hipSetDevice(sim->device));
  if ((rc = sim->upload_hist())) return rc;
  if ((rc = sim->d_sums.ensure(CL_NUM_SUMS))) return rc;
  HIP_TRY(hipMemsetAsync(sim->d_sums.p, 0, CL_NUM_SUMS * sizeof(unsigned long long), sim->stream));
  SumParams p = sim->sum_params();
  p.out = sim->d_sums.p;
  int e = launch_checksums(p, sim->stream);
  if (e) return set_err(CL_E_DEVICE, "checksum kernel launch failed: %s", hipGetErrorString((hipError_t)e));
  unsigned long long h[CL_NUM_SUMS];
  HIP_TRY(hipMemcpyAsync(h, sim->d_sums.p, sizeof h, hipMemcpyDeviceToHost, sim->stream));
  HIP_TRY(hipStreamSynchronize(sim->stream));
  for (int k = 0; k < CL_NUM_SUMS; ++k) out[k] = (int64_t)h[k];
  return CL_OK;
}

int cl_go_delay_schedule(int64_t seed_base, int64_t n, int64_t draws, uint8_t* out) {
  if (!out || n < 0 || draws < 0) return set_err(CL_E_INVALID, "bad arguments");
  go_schedule(seed_base, n, draws, out);
  return CL_OK;
}

int cl_go_int63(int64_t seed, int64_t n, int64_t* out) {
  if (!out || n < 0) return set_err(CL_E_INVALID, "bad arguments");
  GoRand r(seed);
  for (int64_t i = 0; i < n; ++i) out[i] = r.int63();
  return CL_OK;
}

int cl_go_intn(int64_t seed, int32_t bound, int64_t n, int32_t* out) {
  if (!out || n < 0 || bound <= 0) return set_err(CL_E_INVALID, "bad arguments");
  GoRand r(seed);
  for (int64_t i = 0; i < n; ++i) out[i] = r.int31n(bound);
  return CL_OK;
}

}  // extern "C"

// ---- device event trace (logger.go) ------------------------------------------------
int cl_trace_enable(cl_sim* sim, int64_t inst_lo, int32_t n_inst, int32_t cap) {
  SIM_CHECK(sim);
  if (n_inst < 0 || inst_lo < 0 || (n_inst > 0 && (inst_lo + n_inst > sim->n_inst || cap <= 0)))
    return set_err(CL_E_INVALID, "trace range outside the batch");
  sim->trace_lo = inst_lo;
  sim->trace_n = n_inst;
  sim->trace_cap = n_inst > 0 ? cap : 0;
  sim->need_fresh = true;  // the next flush replays the program with the trace build
  return CL_OK;
}

int cl_trace_read(cl_sim* sim, int64_t inst, cl_log_event* out, int32_t cap, int32_t* n_events) {
  SIM_CHECK(sim);
  if (!n_events) return set_err(CL_E_INVALID, "null output");
  if (sim->trace_n <= 0 || inst < sim->trace_lo || inst >= sim->trace_lo + sim->trace_n)
    return set_err(CL_E_INVALID, "instance %lld is not traced", (long long)inst);
  int rc = sim->flush();
  if (rc) return rc;
  const size_t k = (size_t)(inst - sim->trace_lo);
  uint32_t cnt = 0;
  HIP_TRY(hipMemcpy(&cnt, sim->d_trace_cnt.p + k, sizeof cnt, hipMemcpyDeviceToHost));
  const uint32_t have = std::min<uint32_t>(cnt, (uint32_t)sim->trace_cap);
  std::vector<TraceRec> r(have);
  if (have)
    HIP_TRY(hipMemcpy(r.data(), sim->d_trace.p + k * sim->trace_cap, have * sizeof(TraceRec), hipMemcpyDeviceToHost));
  // Logger order: by epoch, then tick deliveries by sender rank, then host events
  std::sort(r.begin(), r.end(), [](const TraceRec& a, const TraceRec& b) {
    const uint64_t ka = ((uint64_t)(a.w0 & 0xffffu) << 32) | a.order, kb = ((uint64_t)(b.w0 & 0xffffu) << 32) | b.order;
    return ka < kb;
  });
  *n_events = (int32_t)have;
  for (uint32_t i = 0; i < have && (int32_t)i < cap && out; ++i) {
    const uint32_t w = r[i].w0, kind = (w >> 16) & 7u, other = w >> 25;
    out[i].epoch = (int32_t)(w & 0xffffu);
    out[i].kind = (int32_t)kind;
    out[i].node = (int32_t)((w >> 19) & 63u);
    out[i].other = (kind == TK_START || kind == TK_END || other == kTraceNoLink) ? -1 : (int32_t)other;
    out[i].data = r[i].data;
    out[i].tokens = r[i].tokens;
  }
  if (cnt > (uint32_t)sim->trace_cap)
    return set_err(CL_E_LIMIT, "trace of instance %lld overflowed: %u records, capacity %d", (long long)inst, cnt,
                   sim->trace_cap);
  return CL_OK;
}
