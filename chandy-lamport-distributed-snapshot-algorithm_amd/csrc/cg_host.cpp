// cg_host.cpp -- host runtime of the graph engine behind include/clgraph.h.
//
// One cl_graph is ONE reference simulation (sim.go ChandyLamportSim) over a topology of
// up to 2^31 nodes / channels whose state lives in HBM:
//   * topology: AddNode/AddLink (or a bulk rank-ordered edge list, or the synthetic
//     generators of SURVEY.md §8(d)) frozen into rank order (getSortedKeys,
//     common.go:135-146): channels by (src rank, dest rank) = out-CSR, plus the in-CSR
//     (dest rank, src rank) that recording cursors are laid out in;
//   * events: SendTokens / StartSnapshot / Tick / drain (sim.go:58-123,
//     test_common.go:79-140) append to a program; flush launches the per-tick kernel
//     sequence of cg_kernels.hip for what is pending, rerun replays it from scratch;
//   * delays: rand.Intn(5) at sim.go:101 is replaced by a pure function of the run's
//     draw index (counter hash, Go math/rand stream, or an explicit schedule), so the
//     reference's draw ORDER decides every delay;
//   * results: snapshots are expanded back into the reference's {tokenMap, messages}
//     shape (sim.go:134-173) from the recording cursors.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <tuple>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/clgraph.h"
#include "cg_engine.h"
#include "cl_text.h"

using namespace clsnap;

namespace {

int gerr(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  const int rc = set_error_v(code, fmt, ap);
  va_end(ap);
  return rc;
}

#define GHIP(expr)                                                                      \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) return gerr(CL_E_DEVICE, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

template <class T>
struct GBuf {
  T* p = nullptr;
  size_t n = 0;
  int ensure(size_t count) {
    if (count == 0) count = 1;
    if (count <= n && p) return CL_OK;
    release();
    GHIP(hipMalloc((void**)&p, count * sizeof(T)));
    n = count;
    return CL_OK;
  }
  int upload(const std::vector<T>& v) {
    int rc = ensure(v.size());
    if (rc) return rc;
    if (!v.empty()) GHIP(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return CL_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  size_t bytes() const { return n * sizeof(T); }
};

// P_HOST: n consecutive host events (gops, in order); P_TICK: n ticks; P_DRAIN: a = snapshots
// started before the drain.
enum ProgKind : int32_t { P_HOST = 1, P_TICK = 3, P_DRAIN = 4 };
struct ProgOp {
  int32_t kind, a, b;
  int64_t n;
};

inline uint64_t mulhi(uint64_t x, uint64_t n) { return (uint64_t)(((unsigned __int128)x * n) >> 64); }

int digits(int64_t x) {
  int d = 1;
  while (x >= 10) {
    x /= 10;
    ++d;
  }
  return d;
}

constexpr int64_t kMaxGraphTime = (1 << 25) - 8;  // pick words hold (tick << 6) | out-index

}  // namespace

struct cl_graph {
  int device = 0;

  // ---- topology ------------------------------------------------------------
  std::vector<std::string> ids;  // insertion order (string mode)
  std::vector<int64_t> init_tokens;
  std::unordered_map<std::string, int> id_index;
  std::vector<std::pair<int, int>> links;
  bool bulk = false;  // ids are "N" + zero-padded rank
  int id_width = 0;
  bool frozen = false;
  int32_t n = 0;
  int64_t e = 0;
  std::vector<int32_t> rank_of, by_rank;
  std::vector<int32_t> out_off, ch_dst, ch_src, ch_inpos, in_off, in_src, init_tok;
  int64_t total_tokens = 0;
  int32_t max_out = 0, max_in = 0;

  // ---- configuration -------------------------------------------------------
  int32_t cap_log2 = 4;
  int32_t max_snaps_cfg = 0;
  int64_t max_drain = 10000;
  int32_t delay_mode = 0;  // 0 hash, 1 schedule (Go seed or explicit)
  uint64_t delay_seed = 0;
  bool go_seed = false;
  int64_t go_seed_val = 0;
  std::vector<uint8_t> user_sched;
  uint64_t traffic_seed = 0;
  uint32_t traffic_thresh = 0;
  int64_t traffic_steps = 0;
  int32_t push_lanes = 0;  // k_push lanes per node: 0 automatic (cl_graph_set_push_lanes)

  // ---- program ---------------------------------------------------------------
  std::vector<ProgOp> prog;
  std::vector<GOp> gops;  // SEND/SNAP ops in program order
  int32_t n_sids = 0;
  int64_t host_sends = 0;
  std::vector<int32_t> ch_sends;  // host sends per channel
  bool nonunit = false;           // a host send moves != 1 token: keep payload history

  // ---- execution -------------------------------------------------------------
  size_t executed = 0;     // program ops executed on the device state
  size_t gop_cursor = 0;   // gops executed
  int64_t time = 0;        // host view of the simulator time
  bool hang = false;
  bool state_valid = false;
  bool dev_ready = false;
  hipStream_t stream = nullptr;      // every launch and copy (cl_graph_set_stream may replace it)
  hipStream_t own_stream = nullptr;  // the engine's own non-blocking stream
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pool;
  size_t ev_used = 0;
  double run_ms = 0;
  int64_t runs = 0, run_ticks = 0, pending_ticks = 0;
  // phases of the latest run (cl_graph_phase_time): start, first drain, end
  hipEvent_t ph_ev[3] = {nullptr, nullptr, nullptr};
  bool ph_drain = false, ph_fresh = false;
  int64_t ph_time[3] = {0, 0, 0};

  GParams P{};
  int32_t s_cap = 0, hist = 0, alloc_cap_log2 = -1;
  int64_t sched_len = 0;
  GBuf<int32_t> d_out_off, d_in_off, d_in_src, d_init_tok;
  GBuf<int2> d_route;
  GBuf<int32_t> d_tokens, d_ltrig, d_lsend, d_crn, d_mcnt;
  GBuf<int2> d_pp;
  GBuf<MDel> d_mlist;
  GBuf<uint32_t> d_tokcnt;
  GBuf<uint8_t> d_in_oj;
  GBuf<BigX> d_big;
  GBuf<unsigned long long> d_cpart;
  GBuf<uint64_t> d_cre;
  GBuf<long long> d_bsum;
  GBuf<uint32_t> d_histv;
  GBuf<uint64_t> d_hq;
  GBuf<uint64_t> d_fifo, d_rec;
  GBuf<SNode> d_sn;
  GBuf<int32_t> d_done, d_ctick;
  GBuf<GScal> d_sc;
  GBuf<GOp> d_ops;
  GBuf<uint8_t> d_sched;
  GBuf<unsigned long long> d_scratch;
  size_t ops_uploaded = 0;
  // device event trace (cl_graph_trace_enable)
  int32_t trace_cap = 0;
  GBuf<GTraceRec> d_trace;
  GBuf<uint32_t> d_trace_cnt;
  // graph-partitioned mode (cl_graph_part_begin)
  bool part = false;
  int32_t part_lo = 0, part_hi = 0;
  GBuf<PDel> d_outbox, d_inbox;
  GBuf<uint32_t> d_out_n;
  GBuf<MDel> d_rmlist;
  GBuf<int2> d_reports, d_rep_in;
  GBuf<int32_t> d_trigv, d_s0;
  GBuf<unsigned long long> d_rdraw, d_draw0;
  GBuf<long long> d_replies;
  GBuf<GOp> d_pop;
  // device-resident exchange (cl_graph_part_dev_bind): caller-owned buckets and totals
  int32_t bk_world = 0, bk_rank = 0, bk_span = 0, bk_cap = 0;
  void *bk_send = nullptr, *bk_recv = nullptr, *tot_send = nullptr, *tot_recv = nullptr;
  GBuf<uint32_t> d_bk_cnt;

  ~cl_graph() {
    if (!dev_ready) return;
    (void)hipSetDevice(device);
    // both streams drain before any buffer is freed: the caller's (cl_graph_set_stream) and
    // the engine's own, which may hold work issued before the switch
    (void)hipStreamSynchronize(stream);
    if (own_stream != stream) (void)hipStreamSynchronize(own_stream);
    GBuf<int32_t>* i32s[] = {&d_out_off, &d_in_off, &d_in_src, &d_init_tok, &d_tokens,
                             &d_ltrig,  &d_lsend,    &d_crn,    &d_mcnt,
                             &d_done,    &d_ctick};
    for (auto* b : i32s) b->release();
    d_cre.release(); d_bsum.release(); d_hq.release(); d_histv.release(); d_mlist.release(); d_route.release();
    d_tokcnt.release(); d_pp.release(); d_in_oj.release(); d_fifo.release(); d_sn.release(); d_rec.release(); d_sc.release(); d_ops.release();
    d_sched.release(); d_scratch.release(); d_big.release(); d_cpart.release();
    d_trace.release(); d_trace_cnt.release();
    d_outbox.release(); d_inbox.release(); d_out_n.release(); d_rmlist.release(); d_reports.release();
    d_rep_in.release(); d_trigv.release(); d_s0.release(); d_rdraw.release(); d_draw0.release();
    d_replies.release(); d_pop.release(); d_bk_cnt.release();
    for (auto& ev : ev_pool) {
      (void)hipEventDestroy(ev.first);
      (void)hipEventDestroy(ev.second);
    }
    for (auto& e : ph_ev)
      if (e) (void)hipEventDestroy(e);
    (void)hipStreamSynchronize(own_stream);
    (void)hipStreamDestroy(own_stream);
  }

  // ---- topology --------------------------------------------------------------
  std::string node_id(int32_t r) const {
    if (bulk) {
      char buf[32];
      snprintf(buf, sizeof buf, "N%0*d", id_width, r);
      return buf;
    }
    return ids[by_rank[r]];
  }

  // rank of an id given as a view (no allocation for ids of up to 15 bytes: std::string SSO)
  int32_t rank_of_sv(std::string_view id) const {
    if (bulk) {
      if (id.size() != (size_t)id_width + 1 || id[0] != 'N') return -1;
      int64_t v = 0;
      for (size_t i = 1; i < id.size(); ++i) {
        if (id[i] < '0' || id[i] > '9') return -1;
        v = v * 10 + (id[i] - '0');
      }
      return v < n ? (int32_t)v : -1;
    }
    auto it = id_index.find(std::string(id));
    if (it == id_index.end()) return -1;
    return frozen ? rank_of[it->second] : it->second;
  }

  // rank of an id, -1 if unknown
  int32_t rank_of_id(const char* id) const {
    if (!id) return -1;
    if (bulk) {
      const size_t L = std::strlen(id);
      if (L != (size_t)id_width + 1 || id[0] != 'N') return -1;
      int64_t v = 0;
      for (size_t i = 1; i < L; ++i) {
        if (id[i] < '0' || id[i] > '9') return -1;
        v = v * 10 + (id[i] - '0');
      }
      return v < n ? (int32_t)v : -1;
    }
    auto it = id_index.find(id);
    if (it == id_index.end()) return -1;
    return frozen ? rank_of[it->second] : it->second;
  }

  // channels (src rank, dst rank), sorted and unique -> CSR
  int build_csr(std::vector<std::pair<int32_t, int32_t>>& ch) {
    std::sort(ch.begin(), ch.end());
    ch.erase(std::unique(ch.begin(), ch.end()), ch.end());
    if (ch.size() >= (size_t)INT32_MAX) return gerr(CL_E_LIMIT, "too many channels");
    e = (int64_t)ch.size();
    out_off.assign(n + 1, 0);
    in_off.assign(n + 1, 0);
    ch_src.resize(e);
    ch_dst.resize(e);
    for (int64_t c = 0; c < e; ++c) {
      ch_src[c] = ch[c].first;
      ch_dst[c] = ch[c].second;
      out_off[ch[c].first + 1]++;
      in_off[ch[c].second + 1]++;
    }
    for (int32_t v = 0; v < n; ++v) {
      out_off[v + 1] += out_off[v];
      in_off[v + 1] += in_off[v];
    }
    ch_inpos.resize(e);
    in_src.resize(e);
    std::vector<int32_t> fill(in_off.begin(), in_off.end() - 1);
    for (int64_t c = 0; c < e; ++c) {  // channels sorted by src: in-lists come out by src rank
      const int32_t k = fill[ch_dst[c]]++;
      ch_inpos[c] = k;
      in_src[k] = ch_src[c];
    }
    max_out = max_in = 0;
    for (int32_t v = 0; v < n; ++v) {
      max_out = std::max(max_out, out_off[v + 1] - out_off[v]);
      max_in = std::max(max_in, in_off[v + 1] - in_off[v]);
    }
    if (max_out > kGMaxOutDegree)
      return gerr(CL_E_LIMIT, "out-degree %d exceeds the graph engine's %d", max_out, kGMaxOutDegree);
    ch_sends.assign(e, 0);
    frozen = true;
    return CL_OK;
  }

  int freeze() {
    if (frozen) return CL_OK;
    n = (int32_t)ids.size();
    by_rank.resize(n);
    std::iota(by_rank.begin(), by_rank.end(), 0);
    std::sort(by_rank.begin(), by_rank.end(), [&](int a, int b) { return ids[a] < ids[b]; });
    rank_of.assign(n, 0);
    for (int r = 0; r < n; ++r) rank_of[by_rank[r]] = r;
    init_tok.resize(n);
    total_tokens = 0;
    for (int r = 0; r < n; ++r) {
      init_tok[r] = (int32_t)init_tokens[by_rank[r]];
      total_tokens += init_tokens[by_rank[r]];
    }
    std::vector<std::pair<int32_t, int32_t>> ch;
    ch.reserve(links.size());
    for (auto& l : links) ch.emplace_back(rank_of[l.first], rank_of[l.second]);
    return build_csr(ch);
  }

  int set_topology(int32_t nn, int32_t width, const int64_t* tokens, int64_t m, const int32_t* src,
                   const int32_t* dst) {
    if (frozen || !ids.empty()) return gerr(CL_E_STATE, "the topology is already set");
    if (nn <= 0 || !tokens || (m > 0 && (!src || !dst)) || m < 0) return gerr(CL_E_INVALID, "bad topology arrays");
    if (width == 0) width = digits(nn - 1);
    if (width < digits(nn - 1) || width > 10)
      return gerr(CL_E_INVALID, "id width %d cannot keep %d ranks in lexicographic order", width, nn);
    n = nn;
    bulk = true;
    id_width = width;
    init_tok.resize(n);
    total_tokens = 0;
    for (int32_t r = 0; r < n; ++r) {
      if (tokens[r] < 0 || tokens[r] > INT32_MAX) return gerr(CL_E_LIMIT, "token count out of range");
      init_tok[r] = (int32_t)tokens[r];
      total_tokens += tokens[r];
    }
    if (total_tokens > INT32_MAX) return gerr(CL_E_LIMIT, "total tokens exceed int32");
    std::vector<std::pair<int32_t, int32_t>> ch;
    ch.reserve((size_t)m);
    for (int64_t i = 0; i < m; ++i) {
      if (src[i] < 0 || src[i] >= n || dst[i] < 0 || dst[i] >= n)
        return gerr(CL_E_UNKNOWN_NODE, "edge %lld references a rank outside [0, %d)", (long long)i, n);
      if (src[i] != dst[i]) ch.emplace_back(src[i], dst[i]);  // node.go:88-90
    }
    return build_csr(ch);
  }

  // ---- program -------------------------------------------------------------------
  int append_send(int32_t a, int32_t b, int64_t nt) {
    if (nt < 0 || nt > (int64_t)kGPayload) return gerr(CL_E_LIMIT, "token count %lld out of range", (long long)nt);
    if (nt != 1) nonunit = true;
    if (b >= 0) {
      // out-index lookup only to count per-channel sends (history sizing)
      auto lo = ch_dst.begin() + out_off[a], hi = ch_dst.begin() + out_off[a + 1];
      auto it = std::lower_bound(lo, hi, b);
      if (it != hi && *it == b) ch_sends[it - ch_dst.begin()]++;
    }
    host_sends++;
    append_host();
    gops.push_back(GOp{GOP_SEND, a, b, (int32_t)nt});
    return CL_OK;
  }

  // one more host event in the program (runs of them share one program op)
  void append_host() {
    if (!prog.empty() && prog.back().kind == P_HOST && executed < prog.size()) {
      prog.back().n += 1;
      return;
    }
    prog.push_back(ProgOp{P_HOST, 0, 0, 1});
  }

  int append_snap(int32_t a, int32_t* out_sid) {
    if (n_sids == INT32_MAX) return gerr(CL_E_LIMIT, "too many snapshots");
    const int32_t sid = n_sids++;
    if (out_sid) *out_sid = sid;
    append_host();
    gops.push_back(GOp{GOP_SNAP, a, sid, 0});
    return CL_OK;
  }

  int append_tick(int64_t k) {
    if (k <= 0) return CL_OK;
    pending_ticks += k;
    if (!prog.empty() && prog.back().kind == P_TICK && executed < prog.size()) {
      prog.back().n += k;
      return CL_OK;
    }
    prog.push_back(ProgOp{P_TICK, 0, 0, k});
    return CL_OK;
  }

  // ---- device ----------------------------------------------------------------------
  int ensure_device() {
    if (dev_ready) return CL_OK;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
      return gerr(CL_E_DEVICE, "no HIP device available (the engine needs a gfx950 GPU)");
    if (device < 0 || device >= count) return gerr(CL_E_DEVICE, "device %d out of range (%d)", device, count);
    GHIP(hipSetDevice(device));
    hipDeviceProp_t prop;
    GHIP(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
      return gerr(CL_E_DEVICE, "device %d is %s, the engine is built for gfx950", device, prop.gcnArchName);
    GHIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    own_stream = stream;
    dev_ready = true;
    int rc;
    std::vector<int2> route((size_t)e);
    for (int64_t c = 0; c < e; ++c) route[c] = make_int2(ch_dst[c], ch_inpos[c]);
    // out-link index at the sender of every in-channel (expansions match it against the
    // sender's delivery word; out-degrees are below 256: kGMaxOutDegree)
    std::vector<uint8_t> in_oj((size_t)e);
    for (int64_t c = 0; c < e; ++c) in_oj[(size_t)ch_inpos[c]] = (uint8_t)(c - out_off[ch_src[c]]);
    if ((rc = d_out_off.upload(out_off)) || (rc = d_route.upload(route)) || (rc = d_in_off.upload(in_off)) ||
        (rc = d_in_src.upload(in_src)) || (rc = d_in_oj.upload(in_oj)) || (rc = d_init_tok.upload(init_tok)))
      return rc;
    return CL_OK;
  }

  int32_t hist_needed() const {
    if (!nonunit) return 0;
    int64_t mx = 0;
    for (auto c : ch_sends) mx = std::max<int64_t>(mx, c);
    mx += traffic_steps;
    int32_t h = 16;
    while (h < mx) h <<= 1;
    return h;
  }

  int64_t draws_bound() const {
    return host_sends + traffic_steps * (int64_t)n + (int64_t)n_sids * e;
  }

  // (Re)allocate the run state when the program outgrew it. Returns 1 in *realloc when
  // the device state was reallocated (the program must then be replayed from the start).
  int ensure_state(bool* reallocated) {
    *reallocated = false;
    const int32_t want_s = std::max({n_sids, max_snaps_cfg, 16});
    const int32_t want_h = hist_needed();
    if (s_cap >= n_sids && hist >= want_h && alloc_cap_log2 == cap_log2 && d_sc.p) return CL_OK;
    *reallocated = true;
    s_cap = std::max(s_cap, want_s);
    hist = std::max(hist, want_h);
    alloc_cap_log2 = cap_log2;
    const size_t N = (size_t)n, E = (size_t)std::max<int64_t>(e, 1);
    const size_t NP = (N + kGThreads - 1) / kGThreads;
    if ((uint64_t)s_cap * N >= (1ull << 40) || (uint64_t)s_cap * E >= (1ull << 40))
      return gerr(CL_E_LIMIT, "snapshot state too large");
    int rc;
    if ((rc = d_tokens.ensure(N)) || (rc = d_pp.ensure(N)) || (rc = d_ltrig.ensure(N)) ||
        (rc = d_lsend.ensure(N)) || (rc = d_crn.ensure(N)) || (rc = d_mlist.ensure(NP * kGThreads)) ||
        (rc = d_mcnt.ensure(NP)) || (rc = d_big.ensure(N)) || (rc = d_cpart.ensure((size_t)kParts * kNumCnt)) ||
        (rc = d_cre.ensure(E)) || (rc = d_bsum.ensure(2 * NP)) || (rc = d_hq.ensure(E)) ||
        (rc = d_tokcnt.ensure(E)) || (rc = d_histv.ensure(hist ? E * hist : 1)) ||
        (rc = d_fifo.ensure(E << cap_log2)) || (rc = d_sn.ensure(s_cap * N)) ||
        (rc = d_rec.ensure(s_cap * E)) ||
        (rc = d_done.ensure((size_t)s_cap * (1 + NP))) || (rc = d_ctick.ensure(s_cap)) || (rc = d_sc.ensure(1)) ||
        (rc = d_scratch.ensure(3 + (size_t)s_cap)))
      return rc;
    return CL_OK;
  }

  int ensure_sched() {
    if (delay_mode == 0) {
      sched_len = 0;
      return CL_OK;
    }
    if (!go_seed) {
      if ((int64_t)d_sched.n >= (int64_t)user_sched.size() && sched_len == (int64_t)user_sched.size()) return CL_OK;
      sched_len = (int64_t)user_sched.size();
      return d_sched.upload(user_sched);
    }
    const int64_t need = std::max<int64_t>(16, draws_bound());
    if (sched_len >= need) return CL_OK;
    std::vector<uint8_t> s((size_t)need);
    int rc = cl_go_delay_schedule(go_seed_val, 1, need, s.data());  // instance 0 of the Go streams
    if (rc) return rc;
    if ((rc = d_sched.upload(s))) return rc;
    sched_len = need;
    return CL_OK;
  }

  void fill_params() {
    GParams& p = P;
    p.n = n;
    p.e = (int32_t)e;
    p.cap_log2 = cap_log2;
    p.s_cap = s_cap;
    p.hist = hist;
    p.delay_mode = delay_mode;
    p.delay_seed = delay_seed;
    p.sched = d_sched.p;
    p.sched_len = sched_len;
    p.traffic_seed = traffic_seed;
    p.traffic_thresh = traffic_thresh;
    p.traffic_steps = traffic_steps;
    p.n_pblocks = (n + kGThreads - 1) / kGThreads;
    p.blk_max_out = 0;
    for (int32_t b = 0; b < p.n_pblocks; ++b)
      p.blk_max_out = std::max(p.blk_max_out, out_off[std::min((int64_t)(b + 1) * kGThreads, (int64_t)n)] - out_off[(int64_t)b * kGThreads]);
    p.push_lanes = push_lanes;
    p.out_off = d_out_off.p;
    p.route = d_route.p;
    p.in_off = d_in_off.p;
    p.in_src = d_in_src.p;
    p.tokens = d_tokens.p;
    p.pp = d_pp.p;
    p.ltrig = d_ltrig.p;
    p.lsend = d_lsend.p;
    p.bsum = d_bsum.p;
    p.crn = d_crn.p;
    p.cre = d_cre.p;
    p.mlist = d_mlist.p;
    p.mcnt = d_mcnt.p;
    p.big = d_big.p;
    p.cpart = d_cpart.p;
    p.hq = d_hq.p;
    p.fifo = d_fifo.p;
    p.tokcnt = d_tokcnt.p;
    p.in_oj = d_in_oj.p;
    p.histv = d_histv.p;
    p.sn = d_sn.p;
    p.rec = d_rec.p;
    p.done = d_done.p;
    p.gdone = d_done.p + s_cap;
    p.ctick = d_ctick.p;
    p.sc = d_sc.p;
    p.ops = d_ops.p;
    p.trace = trace_cap > 0 ? d_trace.p : nullptr;
    p.trace_cnt = trace_cap > 0 ? d_trace_cnt.p : nullptr;
    p.trace_cap = trace_cap;
    p.part = part ? 1 : 0;
    p.part_lo = part ? part_lo : 0;
    p.part_hi = part ? part_hi : n;
    p.blk_lo = p.part_lo / kGThreads;
    p.blk_hi = (p.part_hi + kGThreads - 1) / kGThreads;
    p.outbox = d_outbox.p;
    p.out_n = d_out_n.p;
    p.rmlist = d_rmlist.p;
    p.reports = d_reports.p;
    p.trigv = d_trigv.p;
    p.rdraw = d_rdraw.p;
    p.bk_world = bk_world;
    p.bk_rank = bk_rank;
    p.bk_span = bk_span;
    p.bk_cap = bk_cap;
    p.bk_send = (int4*)bk_send;
    p.bk_recv = (const int4*)bk_recv;
    p.bk_cnt = d_bk_cnt.p;
    p.tot_send = (long long*)tot_send;
    p.tot_recv = (const long long*)tot_recv;
  }

  int upload_ops() {
    if (gops.size() == ops_uploaded && d_ops.p) return CL_OK;
    int rc = d_ops.ensure(std::max<size_t>(gops.size(), 64));
    if (rc) return rc;
    if (!gops.empty()) GHIP(hipMemcpy(d_ops.p, gops.data(), gops.size() * sizeof(GOp), hipMemcpyHostToDevice));
    ops_uploaded = gops.size();
    return CL_OK;
  }

  int k_err(int e_) {
    if (e_) return gerr(CL_E_DEVICE, "graph kernel launch failed: %s", hipGetErrorString((hipError_t)e_));
    return CL_OK;
  }

  int launch_tick() {
    if (time + 1 > kMaxGraphTime) return gerr(CL_E_LIMIT, "simulated time would exceed %lld ticks", (long long)kMaxGraphTime);
    ++time;
    ++run_ticks;
    return k_err(cg_launch_tick(P, (int32_t)time, stream));
  }

  // Host events [pend_begin, +pend_count) in program order.  Maximal runs of at least
  // kSendGroupMin sends from pairwise distinct senders (an event-file step of a large
  // synthetic workload: one send line per node) run as one parallel send group; the rest
  // runs through the sequential k_hostops.
  static constexpr size_t kSendGroupMin = 64;
  std::vector<uint32_t> seen_stamp;
  uint32_t stamp = 0;
  int flush_hostops(size_t& pend_begin, size_t& pend_count) {
    if (!pend_count) return CL_OK;
    int rc = CL_OK;
    const size_t end = pend_begin + pend_count;
    if (seen_stamp.size() != (size_t)n) seen_stamp.assign((size_t)n, 0u);
    size_t i = pend_begin, seq = pend_begin;  // [seq, i): sequential events not yet launched
    while (i < end && rc == CL_OK) {
      size_t j = i;
      if (++stamp == 0) {
        std::fill(seen_stamp.begin(), seen_stamp.end(), 0u);
        stamp = 1;
      }
      while (j < end && gops[j].kind == GOP_SEND && seen_stamp[gops[j].a] != stamp) seen_stamp[gops[j].a] = stamp, ++j;
      if (j - i >= kSendGroupMin) {
        if (i > seq) rc = k_err(cg_launch_hostops(P, (int32_t)time, (int32_t)seq, (int32_t)(i - seq), stream));
        if (rc == CL_OK) rc = k_err(cg_launch_sendgroup(P, (int32_t)time, (int32_t)i, (int32_t)(j - i), stream));
        i = seq = j;
      } else {
        i = std::max(j, i + 1);
      }
    }
    if (rc == CL_OK && end > seq) rc = k_err(cg_launch_hostops(P, (int32_t)time, (int32_t)seq, (int32_t)(end - seq), stream));
    pend_begin = end;
    pend_count = 0;
    return rc;
  }

  int read_status(int32_t* st) {
    GScal sc;
    GHIP(hipMemcpyAsync(&sc, d_sc.p, sizeof sc, hipMemcpyDeviceToHost, stream));
    GHIP(hipStreamSynchronize(stream));
    *st = sc.status;
    return CL_OK;
  }

  // test_common.go:123-137: tick until the snapshots started before this drain (sids
  // [0, n_before)) have completed, then +6.  Later snapshots are not waited for.  The
  // loop runs on the device (k_drain_ctl before every tick decides whether it runs), so
  // the host launches ticks in growing batches and reads the drain state once per batch.
  int run_drain(int32_t n_before) {
    int rc = k_err(cg_launch_drain_begin(P, (int32_t)time, n_before, max_drain, stream));
    if (rc) return rc;
    const int32_t time0 = (int32_t)time;
    int32_t batch = 8;
    int64_t launched = 0;  // drain ticks launched (tick i uses control slot i & 1)
    GScal sc;
    for (;;) {
      if ((rc = k_err(cg_launch_drain_ticks(P, n_before, max_drain, launched, batch, stream)))) return rc;
      launched += batch;
      GHIP(hipMemcpyAsync(&sc, d_sc.p, sizeof sc, hipMemcpyDeviceToHost, stream));
      GHIP(hipStreamSynchronize(stream));
      if (sc.status || sc.dphase == kDrainDone || sc.dphase == kDrainHang) break;
      batch = std::min(batch * 2, 256);
    }
    if (sc.dphase == kDrainHang) hang = true;
    if (!sc.status) time = sc.time;  // (a frozen run reports the device time itself)
    else time = std::max<int64_t>(time, sc.time);
    run_ticks += std::max<int64_t>(0, time - time0);
    return k_err(cg_launch_drain_end(P, stream));
  }

  // Execute program ops [executed, end) on the device; from scratch if `fresh`.
  int run(bool fresh) {
    if (part) return gerr(CL_E_STATE, "a partitioned run advances only through the cl_graph_part_* calls");
    int rc = freeze();
    if (rc) return rc;
    if (n == 0) return gerr(CL_E_STATE, "the topology has no nodes");
    if ((rc = ensure_device())) return rc;
    GHIP(hipSetDevice(device));
    // buffers are only replaced between runs: wait for the previous one first
    if (gops.size() != ops_uploaded || !state_valid) GHIP(hipStreamSynchronize(stream));
    bool realloc = false;
    if ((rc = ensure_state(&realloc))) return rc;
    if ((rc = ensure_sched()) || (rc = upload_ops())) return rc;
    if (trace_cap > 0 && ((rc = d_trace.ensure((size_t)trace_cap)) || (rc = d_trace_cnt.ensure(1)))) return rc;
    fill_params();
    if (realloc || !state_valid) fresh = true;
    if (!fresh && executed == prog.size()) return CL_OK;
    if (ev_used == ev_pool.size()) {
      std::pair<hipEvent_t, hipEvent_t> pr;
      GHIP(hipEventCreateWithFlags(&pr.first, hipEventDisableSystemFence));  // timing only: no cache writeback per record
      GHIP(hipEventCreateWithFlags(&pr.second, hipEventDisableSystemFence));
      ev_pool.push_back(pr);
    }
    auto& ev = ev_pool[ev_used++];
    GHIP(hipEventRecord(ev.first, stream));
    for (auto& e : ph_ev)
      if (!e) GHIP(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    GHIP(hipEventRecord(ph_ev[0], stream));
    ph_drain = false;
    ph_fresh = fresh;
    ph_time[0] = fresh ? 0 : time;
    size_t begin = executed;
    if (fresh) {
      begin = 0;
      gop_cursor = 0;
      time = 0;
      hang = false;
      if ((rc = k_err(cg_launch_reset(P, d_init_tok.p, stream)))) return rc;
      // a replay from the initial state restarts the log (an incremental run appends)
      if (trace_cap > 0) GHIP(hipMemsetAsync(d_trace_cnt.p, 0, sizeof(uint32_t), stream));
      if (traffic_steps > 0 && (rc = k_err(cg_launch_sends(P, 0, stream)))) return rc;  // step 0 traffic
    }
    state_valid = false;
    size_t pend_begin = gop_cursor, pend_count = 0;
    // a HANG freezes the run where the reference's drain would loop forever: later ops
    // never execute (the oracle and the multi-instance engine stop there too)
    for (size_t i = begin; i < prog.size() && !hang; ++i) {
      const ProgOp& op = prog[i];
      if (op.kind == P_HOST) {
        pend_count += (size_t)op.n;
      } else if (op.kind == P_TICK) {
        if ((rc = flush_hostops(pend_begin, pend_count))) return rc;
        for (int64_t k = 0; k < op.n; ++k)
          if ((rc = launch_tick())) return rc;
      } else if (op.kind == P_DRAIN) {
        if ((rc = flush_hostops(pend_begin, pend_count))) return rc;
        if (!ph_drain) {  // the first drain of the run: the traffic / drain phase boundary
          GHIP(hipEventRecord(ph_ev[1], stream));
          ph_drain = true;
          ph_time[1] = time;
        }
        if ((rc = run_drain(op.a))) return rc;
      }
    }
    if ((rc = flush_hostops(pend_begin, pend_count))) return rc;
    GHIP(hipEventRecord(ev.second, stream));
    GHIP(hipEventRecord(ph_ev[2], stream));
    ph_time[2] = time;
    gop_cursor = pend_begin;
    executed = prog.size();
    state_valid = true;
    ++runs;
    return CL_OK;
  }

  // Counter totals: sum of the per-shard partials (cg_engine.h kParts).
  int counter_totals(uint64_t* out) {
    std::vector<unsigned long long> part((size_t)kParts * kNumCnt);
    GHIP(hipMemcpyAsync(part.data(), d_cpart.p, part.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                        stream));
    GHIP(hipStreamSynchronize(stream));
    for (int c = 0; c < kNumCnt; ++c) out[c] = 0;
    for (int sh = 0; sh < kParts; ++sh)
      for (int c = 0; c < kNumCnt; ++c) out[c] += part[(size_t)sh * kNumCnt + c];
    return CL_OK;
  }

  int sync() {
    if (!dev_ready) return CL_OK;
    GHIP(hipSetDevice(device));
    GHIP(hipStreamSynchronize(stream));
    return CL_OK;
  }

  int flush() {
    int rc = CL_OK;
    if (!frozen || !state_valid || executed != prog.size()) rc = run(false);
    if (rc) return rc;
    return sync();
  }

  int fold_time(double* total_ms, int64_t* nruns, int64_t* nticks) {
    int rc = sync();
    if (rc) return rc;
    double ms = 0;
    for (size_t i = 0; i < ev_used; ++i) {
      float f = 0.f;
      GHIP(hipEventElapsedTime(&f, ev_pool[i].first, ev_pool[i].second));
      ms += f;
    }
    ev_used = 0;
    *total_ms = ms;
    *nruns = runs;
    *nticks = run_ticks;
    runs = 0;
    run_ticks = 0;
    return CL_OK;
  }
};

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
#define G_CHECK(g)                                                     \
  do {                                                                 \
    if (!(g)) return gerr(CL_E_INVALID, "null cl_graph handle");       \
  } while (0)
#define G_TOPO_OPEN(g)                                                                       \
  do {                                                                                       \
    if ((g)->frozen) return gerr(CL_E_STATE, "topology changes after events are not supported"); \
  } while (0)

extern "C" {

uint64_t cl_counter_hash(uint64_t seed, uint64_t a, uint64_t b) { return cg_hash(seed, a, b); }

int cl_graph_create(cl_graph** out) {
  if (!out) return gerr(CL_E_INVALID, "null output");
  *out = new cl_graph();
  return CL_OK;
}

int cl_graph_destroy(cl_graph* g) {
  delete g;
  return CL_OK;
}

int cl_graph_set_device(cl_graph* g, int32_t device_ordinal) {
  G_CHECK(g);
  if (g->dev_ready) return gerr(CL_E_STATE, "device already selected");
  g->device = device_ordinal;
  return CL_OK;
}

int cl_graph_add_node(cl_graph* g, const char* id, int64_t tokens) {
  G_CHECK(g);
  G_TOPO_OPEN(g);
  if (g->bulk) return gerr(CL_E_STATE, "bulk topology already set");
  if (!id) return gerr(CL_E_INVALID, "null id");
  if (g->id_index.count(id)) return gerr(CL_E_DUPLICATE_NODE, "node %s already exists", id);
  if (tokens < 0 || tokens > INT32_MAX) return gerr(CL_E_LIMIT, "token count out of range");
  if (g->total_tokens + tokens > INT32_MAX) return gerr(CL_E_LIMIT, "total tokens exceed int32");
  g->total_tokens += tokens;
  g->id_index[id] = (int)g->ids.size();
  g->ids.emplace_back(id);
  g->init_tokens.push_back(tokens);
  return CL_OK;
}

int cl_graph_add_link(cl_graph* g, const char* src, const char* dest) {
  G_CHECK(g);
  const int a = g->rank_of_id(src), b = g->rank_of_id(dest);
  if (a < 0) return gerr(CL_E_UNKNOWN_NODE, "Node %s does not exist", src ? src : "(null)");  // sim.go:49-51
  if (b < 0) return gerr(CL_E_UNKNOWN_NODE, "Node %s does not exist", dest ? dest : "(null)");  // sim.go:52-54
  G_TOPO_OPEN(g);
  if (a != b) g->links.emplace_back(a, b);  // node.go:88-90; duplicates collapse at freeze
  return CL_OK;
}

// readTopologyFile (test_common.go:29-68), streaming over the text without per-line copies:
// lines starting with '#' are comments (:41), the first other line is the node count, the
// next `count` lines "id tokens" are AddNode calls, every later line "src dest" an AddLink.
// The link section -- 8.4M lines for BASELINE config 4 -- is parsed by all host threads
// over newline-aligned chunks (read-only id lookups) and appended in file order; the
// first error in file order is the one reported, as in a sequential parse.
int cl_graph_read_topology_text(cl_graph* g, const char* text) {
  G_CHECK(g);
  if (!text) return gerr(CL_E_INVALID, "null text");
  const std::string_view all(text);
  LineIter it{all};
  std::string_view line, f[3];
  int64_t left = -1;
  size_t link_start = all.size();
  while (it.next(&line)) {
    if (line[0] == '#') continue;
    if (left < 0) {
      if (!go_atoi_sv(line, &left)) return gerr(CL_E_PARSE, "bad node count line: %.*s", (int)line.size(), line.data());
      if (left == 0) {
        link_start = it.i;
        break;
      }
      continue;
    }
    if (go_fields_sv(line, f, 3) != 2)
      return gerr(CL_E_PARSE, "Expected 2 tokens in line: %.*s", (int)line.size(), line.data());
    int64_t tok;
    if (!go_atoi_sv(f[1], &tok)) return gerr(CL_E_PARSE, "bad token count: %.*s", (int)f[1].size(), f[1].data());
    int rc = cl_graph_add_node(g, std::string(f[0]).c_str(), tok);
    if (rc) return rc;
    if (--left == 0) {
      link_start = it.i;
      break;
    }
  }
  if (link_start >= all.size()) return CL_OK;
  if (g->frozen) return gerr(CL_E_STATE, "topology changes after events are not supported");
  // ---- the link section, in parallel ----
  const std::string_view rest = all.substr(link_start);
  const int T = (int)std::max<size_t>(1, std::min<size_t>(std::max(1u, std::thread::hardware_concurrency()),
                                                           rest.size() / (1 << 20) + 1));
  std::vector<size_t> cut(T + 1, rest.size());
  cut[0] = 0;
  for (int t = 1; t < T; ++t) {  // chunk boundaries just after a newline
    size_t c = rest.size() * t / T;
    const size_t nl = rest.find('\n', c);
    cut[t] = nl == std::string_view::npos ? rest.size() : nl + 1;
    if (cut[t] < cut[t - 1]) cut[t] = cut[t - 1];
  }
  struct Part {
    std::vector<std::pair<int, int>> links;
    size_t err_pos = SIZE_MAX;
    int err_code = 0;
    std::string err;
  };
  std::vector<Part> parts(T);
  auto lookup = [&](std::string_view id) -> int {
    auto f2 = g->id_index.find(std::string(id));
    return f2 == g->id_index.end() ? -1 : f2->second;
  };
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      Part& P = parts[t];
      LineIter li{rest.substr(0, cut[t + 1]), cut[t]};
      std::string_view ln, ff[3];
      while (li.next(&ln)) {
        if (ln[0] == '#') continue;
        const size_t pos = (size_t)(ln.data() - rest.data());
        if (go_fields_sv(ln, ff, 3) != 2) {
          P.err_pos = pos, P.err_code = CL_E_PARSE, P.err = "Expected 2 tokens in line: " + std::string(ln);
          return;
        }
        const int a = lookup(ff[0]), b = a < 0 ? -1 : lookup(ff[1]);
        if (a < 0 || b < 0) {  // sim.go:49-54 log.Fatalf("Node %v does not exist")
          P.err_pos = pos, P.err_code = CL_E_UNKNOWN_NODE;
          P.err = "Node " + std::string(a < 0 ? ff[0] : ff[1]) + " does not exist";
          return;
        }
        if (a != b) P.links.emplace_back(a, b);  // node.go:88-90
      }
    });
  for (auto& x : th) x.join();
  for (int t = 0; t < T; ++t) {  // file order: links of earlier chunks, then the first error
    g->links.insert(g->links.end(), parts[t].links.begin(), parts[t].links.end());
    if (parts[t].err_code) return gerr(parts[t].err_code, "%s", parts[t].err.c_str());
  }
  return CL_OK;
}

int cl_graph_read_topology_file(cl_graph* g, const char* path) {
  G_CHECK(g);
  std::string text;
  if (!path || !read_file(path, &text)) return gerr(CL_E_IO, "cannot read %s", path ? path : "(null)");
  return cl_graph_read_topology_text(g, text.c_str());
}

int cl_graph_set_topology(cl_graph* g, int32_t n_nodes, int32_t id_width, const int64_t* tokens, int64_t n_edges,
                          const int32_t* src, const int32_t* dst) {
  G_CHECK(g);
  return g->set_topology(n_nodes, id_width, tokens, n_edges, src, dst);
}

int cl_graph_generate_regular(cl_graph* g, int32_t n_nodes, int32_t degree, int64_t tokens, uint64_t seed) {
  G_CHECK(g);
  if (n_nodes <= 0 || degree < 0 || degree > kGMaxOutDegree) return gerr(CL_E_INVALID, "bad regular graph size");
  const size_t N = (size_t)n_nodes;
  std::vector<int32_t> src(N * degree), dst(N * degree);
  std::vector<std::thread> th;
  for (int p = 0; p < degree; ++p) {
    th.emplace_back([&, p] {
      std::vector<int32_t> perm(N);
      std::iota(perm.begin(), perm.end(), 0);
      for (size_t i = N - 1; i >= 1; --i) {  // Fisher-Yates
        const size_t j = (size_t)mulhi(cg_hash(seed, (uint64_t)p, (uint64_t)i), (uint64_t)(i + 1));
        std::swap(perm[i], perm[j]);
      }
      for (size_t v = 0; v < N; ++v) {
        src[(size_t)p * N + v] = (int32_t)v;
        dst[(size_t)p * N + v] = perm[v];
      }
    });
  }
  for (auto& t : th) t.join();
  std::vector<int64_t> tok(N, tokens);
  return g->set_topology(n_nodes, 0, tok.data(), (int64_t)src.size(), src.data(), dst.data());
}

int cl_graph_generate_powerlaw(cl_graph* g, int32_t n_nodes, int32_t targets, double exponent, int32_t ring,
                               int64_t tokens, uint64_t seed) {
  G_CHECK(g);
  if (n_nodes <= 0 || targets < 0 || targets > kGMaxOutDegree - 2) return gerr(CL_E_INVALID, "bad power-law graph size");
  const size_t N = (size_t)n_nodes;
  std::vector<double> cdf(N);
  double acc = 0;
  for (size_t k = 0; k < N; ++k) {
    acc += std::pow((double)(k + 1), -exponent);
    cdf[k] = acc;
  }
  const double total = acc;
  std::vector<int32_t> src, dst;
  src.reserve(N * (targets + 2));
  dst.reserve(N * (targets + 2));
  for (size_t v = 0; v < N; ++v) {
    for (int i = 0; i < targets; ++i) {
      const uint64_t u = cg_hash(seed, (uint64_t)v, (uint64_t)i);
      const double r = (double)(u >> 11) * (1.0 / 9007199254740992.0) * total;
      size_t k = (size_t)(std::upper_bound(cdf.begin(), cdf.end(), r) - cdf.begin());
      if (k >= N) k = N - 1;
      src.push_back((int32_t)v);
      dst.push_back((int32_t)k);
    }
  }
  if (ring) {
    for (size_t v = 0; v < N; ++v) {
      src.push_back((int32_t)v);
      dst.push_back((int32_t)((v + 1) % N));
      src.push_back((int32_t)v);
      dst.push_back((int32_t)((v + N - 1) % N));
    }
  }
  std::vector<int64_t> tok(N, tokens);
  return g->set_topology(n_nodes, 0, tok.data(), (int64_t)src.size(), src.data(), dst.data());
}

int cl_graph_num_nodes(cl_graph* g, int32_t* n) {
  G_CHECK(g);
  if (!n) return gerr(CL_E_INVALID, "null output");
  int rc = g->freeze();
  if (rc) return rc;
  *n = g->n;
  return CL_OK;
}

int cl_graph_num_channels(cl_graph* g, int64_t* n) {
  G_CHECK(g);
  if (!n) return gerr(CL_E_INVALID, "null output");
  int rc = g->freeze();
  if (rc) return rc;
  *n = g->e;
  return CL_OK;
}

int cl_graph_channels(cl_graph* g, int32_t* src, int32_t* dst) {
  G_CHECK(g);
  int rc = g->freeze();
  if (rc) return rc;
  if (src) std::copy(g->ch_src.begin(), g->ch_src.end(), src);
  if (dst) std::copy(g->ch_dst.begin(), g->ch_dst.end(), dst);
  return CL_OK;
}

int cl_graph_node_id(cl_graph* g, int32_t rank, char* buf, int32_t cap) {
  G_CHECK(g);
  int rc = g->freeze();
  if (rc) return rc;
  if (rank < 0 || rank >= g->n || !buf || cap <= 0) return gerr(CL_E_INVALID, "bad rank or buffer");
  const std::string s = g->node_id(rank);
  if ((int32_t)s.size() >= cap) return gerr(CL_E_LIMIT, "buffer too small");
  std::memcpy(buf, s.c_str(), s.size() + 1);
  return CL_OK;
}

int cl_graph_set_limits(cl_graph* g, int32_t fifo_slots, int32_t max_snapshots, int64_t max_drain_ticks) {
  G_CHECK(g);
  int l = 0;
  while ((1 << l) < fifo_slots) ++l;
  if (fifo_slots < 2 || fifo_slots > 32768 || (1 << l) != fifo_slots)
    return gerr(CL_E_INVALID, "fifo_slots must be a power of two in [2, 32768]");
  if (max_snapshots < 0 || max_drain_ticks < 0) return gerr(CL_E_INVALID, "negative limit");
  if (l != g->cap_log2) g->state_valid = false;
  g->cap_log2 = l;
  g->max_snaps_cfg = max_snapshots;
  g->max_drain = max_drain_ticks;
  return CL_OK;
}

int cl_graph_set_push_lanes(cl_graph* g, int32_t lanes) {
  G_CHECK(g);
  if (lanes != 0 && lanes != 1 && lanes != kPushLanes)
    return gerr(CL_E_INVALID, "push lanes must be 0 (automatic), 1 or %d", kPushLanes);
  g->push_lanes = lanes;
  return CL_OK;
}

int cl_graph_node_id_length(cl_graph* g, int32_t rank, int32_t* len) {
  G_CHECK(g);
  int rc = g->freeze();
  if (rc) return rc;
  if (rank < 0 || rank >= g->n || !len) return gerr(CL_E_INVALID, "bad rank or output");
  *len = (int32_t)g->node_id(rank).size();
  return CL_OK;
}

int cl_graph_set_delay_hash(cl_graph* g, uint64_t seed) {
  G_CHECK(g);
  g->delay_mode = 0;
  g->delay_seed = seed;
  g->go_seed = false;
  g->state_valid = false;
  return CL_OK;
}

int cl_graph_set_delay_go_seed(cl_graph* g, int64_t seed) {
  G_CHECK(g);
  g->delay_mode = 1;
  g->go_seed = true;
  g->go_seed_val = seed;
  g->sched_len = 0;
  g->state_valid = false;
  return CL_OK;
}

int cl_graph_set_delay_schedule(cl_graph* g, const uint8_t* delays, int64_t n) {
  G_CHECK(g);
  if (!delays || n <= 0) return gerr(CL_E_INVALID, "empty schedule");
  for (int64_t i = 0; i < n; ++i)
    if (delays[i] >= 5) return gerr(CL_E_INVALID, "delay %u at %lld outside [0, maxDelay)", delays[i], (long long)i);
  g->user_sched.assign(delays, delays + n);
  g->delay_mode = 1;
  g->go_seed = false;
  g->sched_len = -1;
  g->state_valid = false;
  return CL_OK;
}

int cl_graph_set_traffic(cl_graph* g, uint64_t seed, uint32_t threshold, int64_t steps) {
  G_CHECK(g);
  if (steps < 0) return gerr(CL_E_INVALID, "negative traffic steps");
  g->traffic_seed = seed;
  g->traffic_thresh = threshold;
  g->traffic_steps = threshold ? steps : 0;
  g->state_valid = false;
  return CL_OK;
}

int cl_graph_send_tokens_rank(cl_graph* g, int32_t src, int32_t dest, int64_t n) {
  G_CHECK(g);
  int rc = g->freeze();
  if (rc) return rc;
  if (src < 0 || src >= g->n) return gerr(CL_E_UNKNOWN_NODE, "send from unknown rank %d", src);
  return g->append_send(src, dest >= 0 && dest < g->n ? dest : -1, n);
}

int cl_graph_send_tokens(cl_graph* g, const char* src, const char* dest, int64_t n) {
  G_CHECK(g);
  int rc = g->freeze();
  if (rc) return rc;
  const int32_t a = g->rank_of_id(src);
  if (a < 0) return gerr(CL_E_UNKNOWN_NODE, "send from unknown node %s", src ? src : "(null)");
  return g->append_send(a, g->rank_of_id(dest), n);  // unknown dest: fatal at run time (node.go:121-124)
}

int cl_graph_start_snapshot_rank(cl_graph* g, int32_t node, int32_t* out_sid) {
  G_CHECK(g);
  int rc = g->freeze();
  if (rc) return rc;
  if (node < 0 || node >= g->n) return gerr(CL_E_UNKNOWN_NODE, "snapshot at unknown rank %d", node);
  return g->append_snap(node, out_sid);
}

int cl_graph_start_snapshot(cl_graph* g, const char* node, int32_t* out_sid) {
  G_CHECK(g);
  int rc = g->freeze();
  if (rc) return rc;
  const int32_t a = g->rank_of_id(node);
  if (a < 0) return gerr(CL_E_UNKNOWN_NODE, "snapshot at unknown node %s", node ? node : "(null)");
  return g->append_snap(a, out_sid);
}

int cl_graph_tick(cl_graph* g, int32_t n) {
  G_CHECK(g);
  int rc = g->freeze();
  if (rc) return rc;
  return g->append_tick(n);
}

int cl_graph_drain(cl_graph* g) {
  G_CHECK(g);
  int rc = g->freeze();
  if (rc) return rc;
  g->prog.push_back(ProgOp{P_DRAIN, g->n_sids, 0, 0});  // waits for the snapshots started so far
  return CL_OK;
}

// readEventsFile (test_common.go:79-140) incl. the drain, streaming over the text: the
// event lines of a large synthetic workload (one `send` line per sending node and step)
// append to the program without per-line copies; runs of sends from distinct senders
// execute as parallel send groups (cg_launch_sendgroup).
int cl_graph_read_events_text(cl_graph* g, const char* text, int32_t* n_snapshots) {
  G_CHECK(g);
  if (!text) return gerr(CL_E_INVALID, "null text");
  int rc = g->freeze();
  if (rc) return rc;
  int32_t snaps = 0;
  LineIter it{std::string_view(text)};
  std::string_view line, f[4];
  while (it.next(&line)) {
    if (line == "#") continue;  // strings.HasPrefix("#", line) (test_common.go:90, sic)
    const int nf = go_fields_sv(line, f, 4);
    if (nf == 0) return gerr(CL_E_PARSE, "empty event line");
    if (f[0] == "send") {
      int64_t nt;
      if (nf < 4 || !go_atoi_sv(f[3], &nt)) return gerr(CL_E_PARSE, "bad send line: %.*s", (int)line.size(), line.data());
      const int32_t a = g->rank_of_sv(f[1]);
      if (a < 0) return gerr(CL_E_UNKNOWN_NODE, "send from unknown node %.*s", (int)f[1].size(), f[1].data());
      rc = g->append_send(a, g->rank_of_sv(f[2]), nt);  // unknown dest: fatal at run time (node.go:121-124)
    } else if (f[0] == "snapshot") {
      if (nf < 2) return gerr(CL_E_PARSE, "bad snapshot line: %.*s", (int)line.size(), line.data());
      snaps++;
      const int32_t a = g->rank_of_sv(f[1]);
      if (a < 0) return gerr(CL_E_UNKNOWN_NODE, "snapshot at unknown node %.*s", (int)f[1].size(), f[1].data());
      rc = g->append_snap(a, nullptr);
    } else if (f[0] == "tick") {
      int64_t nt = 1;
      if (nf > 1 && !go_atoi_sv(f[1], &nt)) return gerr(CL_E_PARSE, "bad tick line: %.*s", (int)line.size(), line.data());
      if (nt > INT32_MAX) return gerr(CL_E_LIMIT, "tick count too large");
      rc = g->append_tick(std::max<int64_t>(nt, 0));
    } else {
      return gerr(CL_E_PARSE, "Unknown event command: %.*s", (int)f[0].size(), f[0].data());
    }
    if (rc) return rc;
  }
  if (n_snapshots) *n_snapshots = snaps;
  return cl_graph_drain(g);
}

int cl_graph_read_events_file(cl_graph* g, const char* path, int32_t* n_snapshots) {
  G_CHECK(g);
  std::string text;
  if (!path || !read_file(path, &text)) return gerr(CL_E_IO, "cannot read %s", path ? path : "(null)");
  return cl_graph_read_events_text(g, text.c_str(), n_snapshots);
}

int cl_graph_flush(cl_graph* g) {
  G_CHECK(g);
  return g->flush();
}

int cl_graph_rerun(cl_graph* g) {
  G_CHECK(g);
  return g->run(true);
}

int cl_graph_synchronize(cl_graph* g) {
  G_CHECK(g);
  return g->sync();
}

int cl_graph_run_time(cl_graph* g, double* total_ms, int64_t* runs, int64_t* ticks) {
  G_CHECK(g);
  if (!total_ms || !runs || !ticks) return gerr(CL_E_INVALID, "null output");
  return g->fold_time(total_ms, runs, ticks);
}

int cl_graph_debug_poison_outputs(cl_graph* g) {
  G_CHECK(g);
  if (!g->dev_ready || !g->d_tokens.p) return CL_OK;
  GHIP(hipSetDevice(g->device));
  GHIP(hipMemsetAsync(g->d_tokens.p, 0xA5, g->d_tokens.bytes(), g->stream));
  // (the whole record plane: the run's reset rewrites W and cnt, so stok stays poisoned
  // wherever the run creates no local snapshot)
  GHIP(hipMemsetAsync(g->d_sn.p, 0xA5, g->d_sn.bytes(), g->stream));
  GHIP(hipMemsetAsync(g->d_rec.p, 0xA5, g->d_rec.bytes(), g->stream));
  GHIP(hipMemsetAsync(g->d_ctick.p, 0xA5, g->d_ctick.bytes(), g->stream));
  GHIP(hipMemsetAsync(g->d_cpart.p, 0xA5, g->d_cpart.bytes(), g->stream));
  return CL_OK;
}

int cl_graph_phase_time(cl_graph* g, double* ms, int64_t* ticks) {
  G_CHECK(g);
  if (!ms || !ticks) return gerr(CL_E_INVALID, "null output");
  if (!g->ph_ev[2]) return gerr(CL_E_STATE, "nothing has run");
  int rc = g->sync();
  if (rc) return rc;
  float a = 0.f, b = 0.f;
  if (g->ph_drain) {
    GHIP(hipEventElapsedTime(&a, g->ph_ev[0], g->ph_ev[1]));
    GHIP(hipEventElapsedTime(&b, g->ph_ev[1], g->ph_ev[2]));
    ticks[0] = g->ph_time[1] - g->ph_time[0];
    ticks[1] = g->ph_time[2] - g->ph_time[1];
  } else {
    GHIP(hipEventElapsedTime(&a, g->ph_ev[0], g->ph_ev[2]));
    ticks[0] = g->ph_time[2] - g->ph_time[0];
    ticks[1] = 0;
  }
  ms[0] = a;
  ms[1] = b;
  return CL_OK;
}

int cl_graph_device_bytes(cl_graph* g, int64_t* bytes) {
  G_CHECK(g);
  if (!bytes) return gerr(CL_E_INVALID, "null output");
  size_t b = 0;
  b += g->d_out_off.bytes() + g->d_route.bytes() + g->d_in_off.bytes() +
       g->d_in_src.bytes() + g->d_init_tok.bytes() + g->d_tokens.bytes() + g->d_pp.bytes() + g->d_tokcnt.bytes() + g->d_in_oj.bytes() +
       g->d_ltrig.bytes() + g->d_lsend.bytes() + g->d_crn.bytes() + g->d_mlist.bytes() + g->d_mcnt.bytes() +
       g->d_big.bytes() + g->d_cpart.bytes() +
       g->d_cre.bytes() + g->d_bsum.bytes() + g->d_hq.bytes() +
       g->d_histv.bytes() + g->d_fifo.bytes() + g->d_sn.bytes() + g->d_rec.bytes() + g->d_done.bytes() + g->d_ctick.bytes() + g->d_sched.bytes();
  *bytes = (int64_t)b;
  return CL_OK;
}

int cl_graph_get_status(cl_graph* g, int32_t* status) {
  G_CHECK(g);
  if (!status) return gerr(CL_E_INVALID, "null output");
  int rc = g->flush();
  if (rc) return rc;
  if ((rc = g->read_status(status))) return rc;
  if (!*status && g->hang) *status = CL_INST_HANG;
  return CL_OK;
}

int cl_graph_get_time(cl_graph* g, int64_t* time) {
  G_CHECK(g);
  if (!time) return gerr(CL_E_INVALID, "null output");
  int rc = g->flush();
  if (rc) return rc;
  GScal sc;
  GHIP(hipMemcpy(&sc, g->d_sc.p, sizeof sc, hipMemcpyDeviceToHost));
  *time = sc.status ? sc.time : g->time;
  return CL_OK;
}

int cl_graph_num_snapshots(cl_graph* g, int32_t* n) {
  G_CHECK(g);
  if (!n) return gerr(CL_E_INVALID, "null output");
  *n = g->n_sids;
  return CL_OK;
}

int cl_graph_node_tokens(cl_graph* g, int64_t* out) {
  G_CHECK(g);
  if (!out) return gerr(CL_E_INVALID, "null output");
  int rc = g->flush();
  if (rc) return rc;
  std::vector<int32_t> t((size_t)g->n);
  GHIP(hipMemcpy(t.data(), g->d_tokens.p, t.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
  for (size_t i = 0; i < t.size(); ++i) out[i] = t[i];
  return CL_OK;
}

int cl_graph_snapshot_tick(cl_graph* g, int32_t sid, int32_t* tick) {
  G_CHECK(g);
  if (!tick) return gerr(CL_E_INVALID, "null output");
  if (sid < 0 || sid >= g->n_sids) return gerr(CL_E_INVALID, "unknown snapshot %d", sid);
  int rc = g->flush();
  if (rc) return rc;
  GHIP(hipMemcpy(tick, g->d_ctick.p + sid, sizeof(int32_t), hipMemcpyDeviceToHost));
  return CL_OK;
}

int cl_graph_collect_snapshot(cl_graph* g, int32_t sid, int64_t* tokens, int64_t* msg_offsets, int64_t* msg_tokens,
                              int64_t msg_cap) {
  G_CHECK(g);
  if (sid < 0 || sid >= g->n_sids) return gerr(CL_E_INVALID, "unknown snapshot %d", sid);
  int32_t tick;
  int rc = cl_graph_snapshot_tick(g, sid, &tick);
  if (rc) return rc;
  if (tick < 0) return gerr(CL_E_NOT_COMPLETE, "snapshot %d has not completed", sid);
  const size_t N = (size_t)g->n, E = (size_t)g->e;
  if (tokens) {
    std::vector<int32_t> st(N);
    // (the stok word of each 16-byte record of the plane: one strided copy)
    GHIP(hipMemcpy2D(st.data(), sizeof(int32_t), &g->d_sn.p[(size_t)sid * N].stok, sizeof(SNode), sizeof(int32_t), N,
                     hipMemcpyDeviceToHost));
    for (size_t v = 0; v < N; ++v) tokens[v] = st[v];
  }
  if (!msg_offsets) return CL_OK;
  std::vector<uint64_t> rec(E);
  if (E) GHIP(hipMemcpy(rec.data(), g->d_rec.p + (size_t)sid * E, E * sizeof(uint64_t), hipMemcpyDeviceToHost));
  int64_t m = 0;
  for (size_t c = 0; c < E; ++c) {
    const uint64_t x = rec[g->ch_inpos[c]];
    msg_offsets[c] = m;
    m += (int64_t)((uint32_t)(x >> 32) - (uint32_t)x);
  }
  msg_offsets[E] = m;
  if (m > msg_cap || (m > 0 && !msg_tokens)) return gerr(CL_E_LIMIT, "%lld messages exceed msg_cap", (long long)m);
  std::vector<uint32_t> hv;
  if (g->hist && m) {
    hv.resize(E * (size_t)g->hist);
    GHIP(hipMemcpy(hv.data(), g->d_histv.p, hv.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
  }
  for (size_t c = 0; c < E; ++c) {
    const size_t k = (size_t)g->ch_inpos[c];
    const uint64_t x = rec[k];
    const uint32_t b = (uint32_t)x, e = (uint32_t)(x >> 32);
    for (uint32_t q = b; q < e; ++q)
      msg_tokens[msg_offsets[c] + (q - b)] = g->hist ? (int64_t)hv[k * g->hist + q] : 1;
  }
  return CL_OK;
}

int cl_graph_trace_enable(cl_graph* g, int32_t capacity) {
  G_CHECK(g);
  if (capacity < 0) return gerr(CL_E_INVALID, "negative trace capacity");
  g->trace_cap = capacity;
  g->state_valid = false;  // the next flush replays the program with tracing on (or off)
  return CL_OK;
}

int cl_graph_trace_read(cl_graph* g, cl_log_event* out, int32_t cap, int32_t* n_events) {
  G_CHECK(g);
  if (!n_events) return gerr(CL_E_INVALID, "null output");
  if (g->trace_cap <= 0) return gerr(CL_E_INVALID, "tracing is off (cl_graph_trace_enable)");
  int rc = g->flush();
  if (rc) return rc;
  uint32_t cnt = 0;
  GHIP(hipMemcpy(&cnt, g->d_trace_cnt.p, sizeof cnt, hipMemcpyDeviceToHost));
  const uint32_t have = std::min<uint32_t>(cnt, (uint32_t)g->trace_cap);
  std::vector<GTraceRec> r(have);
  if (have) GHIP(hipMemcpy(r.data(), g->d_trace.p, have * sizeof(GTraceRec), hipMemcpyDeviceToHost));
  if (cnt > (uint32_t)g->trace_cap)
    return gerr(CL_E_LIMIT, "trace overflowed: %u records, capacity %d", cnt, g->trace_cap);
  // EndSnapshotRecord (sim.go:127) follows the delivery that completed the local snapshot:
  // the last marker of that snapshot delivered to the node in that tick, in sender order
  // (the device counts completions in whatever order the atomics land).
  std::map<std::tuple<int32_t, int32_t, int32_t>, uint32_t> last;
  for (const auto& x : r)
    if (x.kind == TK_RECV_MARKER && (x.order >> 30) == kTrTick) {
      auto& l = last[std::make_tuple(x.epoch, x.node, x.data)];
      l = std::max(l, x.order & 0x3fffffffu);
    }
  for (auto& x : r)
    if (x.kind == TK_END) x.order = (kTrTick << 30) | last[std::make_tuple(x.epoch, x.node, x.data)];
  std::sort(r.begin(), r.end(), [](const GTraceRec& a, const GTraceRec& b) {
    return std::make_tuple(a.epoch, a.order, a.sub) < std::make_tuple(b.epoch, b.order, b.sub);
  });
  // LogEvent.nodeTokens (logger.go:71-76): the node's tokens when the record is made --
  // replayed from the initial tokens through the token changes the records carry
  std::vector<int64_t> tok(g->init_tok.begin(), g->init_tok.end());
  *n_events = (int32_t)have;
  for (uint32_t i = 0; i < have; ++i) {
    const GTraceRec& x = r[i];
    if (out && (int32_t)i < cap) {
      out[i].epoch = x.epoch;
      out[i].kind = x.kind;
      out[i].node = x.node;
      out[i].other = x.other;
      out[i].data = x.data;
      out[i].tokens = (int32_t)tok[x.node];
    }
    if (x.kind == TK_SENT_TOKEN) tok[x.node] -= x.data;       // node.go:118-120
    else if (x.kind == TK_RECV_TOKEN) tok[x.node] += x.data;  // node.go:175
  }
  return CL_OK;
}

int cl_graph_get_counters(cl_graph* g, int64_t* out) {
  G_CHECK(g);
  if (!out) return gerr(CL_E_INVALID, "null output");
  int rc = g->flush();
  if (rc) return rc;
  GHIP(hipMemsetAsync(g->d_scratch.p, 0, sizeof(unsigned long long), g->stream));
  if ((rc = g->k_err(cg_launch_finish(g->P, g->n_sids, g->d_scratch.p, g->stream)))) return rc;
  GScal sc;
  unsigned long long open = 0;
  uint64_t cnt[kNumCnt];
  if ((rc = g->counter_totals(cnt))) return rc;
  GHIP(hipMemcpyAsync(&sc, g->d_sc.p, sizeof sc, hipMemcpyDeviceToHost, g->stream));
  GHIP(hipMemcpyAsync(&open, g->d_scratch.p, sizeof open, hipMemcpyDeviceToHost, g->stream));
  GHIP(hipStreamSynchronize(g->stream));
  out[CL_CNT_PUSH] = (int64_t)cnt[GC_PUSH];
  out[CL_CNT_PEEK] = (int64_t)cnt[GC_PEEK];
  out[CL_CNT_POP_TOKEN] = (int64_t)cnt[GC_POP_TOK];
  out[CL_CNT_POP_MARKER] = (int64_t)cnt[GC_POP_MK];
  out[CL_CNT_RECORDED] = (int64_t)open;  // (k_finish: every created local snapshot's recorded copies)
  out[CL_CNT_COMPLETED] = (int64_t)cnt[GC_COMPLETED];
  out[CL_CNT_INSTANCES] = 1;
  out[CL_CNT_TICKS] = sc.status ? sc.time : g->time;
  return CL_OK;
}

int cl_graph_get_checksums(cl_graph* g, int64_t* out) {
  G_CHECK(g);
  if (!out) return gerr(CL_E_INVALID, "null output");
  int rc = g->flush();
  if (rc) return rc;
  const size_t ns = 3 + (size_t)g->n_sids;
  GHIP(hipMemsetAsync(g->d_scratch.p, 0, ns * sizeof(unsigned long long), g->stream));
  if ((rc = g->k_err(cg_launch_checks(g->P, g->n_sids, g->d_scratch.p, g->stream)))) return rc;
  std::vector<unsigned long long> r(ns);
  std::vector<int32_t> ct((size_t)std::max(g->n_sids, 1));
  GScal sc;
  GHIP(hipMemcpyAsync(r.data(), g->d_scratch.p, ns * sizeof(unsigned long long), hipMemcpyDeviceToHost, g->stream));
  if (g->n_sids)
    GHIP(hipMemcpyAsync(ct.data(), g->d_ctick.p, (size_t)g->n_sids * sizeof(int32_t), hipMemcpyDeviceToHost, g->stream));
  GHIP(hipMemcpyAsync(&sc, g->d_sc.p, sizeof sc, hipMemcpyDeviceToHost, g->stream));
  GHIP(hipStreamSynchronize(g->stream));
  int64_t cut = 0, completed = 0;
  for (int32_t s = 0; s < g->n_sids; ++s) {
    if (ct[s] < 0) continue;
    completed++;
    const int64_t d = (int64_t)r[3 + s] - g->total_tokens;
    cut += d < 0 ? -d : d;
  }
  const int64_t fin = (int64_t)r[0] + (int64_t)r[1] - g->total_tokens;
  out[CL_GSUM_OK] = (sc.status == 0 && !g->hang) ? 1 : 0;
  uint64_t cnt[kNumCnt];
  if ((rc = g->counter_totals(cnt))) return rc;
  out[CL_GSUM_DELIVERED] = (int64_t)(cnt[GC_POP_TOK] + cnt[GC_POP_MK]);
  out[CL_GSUM_COMPLETED] = completed;
  out[CL_GSUM_CUT_RESIDUAL] = cut;
  out[CL_GSUM_FINAL_RESIDUAL] = fin < 0 ? -fin : fin;
  out[CL_GSUM_DIGEST] = (int64_t)r[2];
  out[CL_GSUM_IN_FLIGHT] = (int64_t)r[1];
  return CL_OK;
}

// ---- graph-partitioned mode ---------------------------------------------
#define G_PART(g)                                                                            \
  do {                                                                                       \
    if (!(g)->part) return gerr(CL_E_STATE, "not a partitioned run (cl_graph_part_begin)");  \
  } while (0)

int cl_graph_part_begin(cl_graph* g, int32_t node_lo, int32_t node_hi) {
  G_CHECK(g);
  int rc = g->freeze();
  if (rc) return rc;
  if (g->part) return gerr(CL_E_STATE, "the partitioned run has begun");
  if (!g->prog.empty()) return gerr(CL_E_STATE, "a partitioned run starts from an empty program");
  if (g->trace_cap > 0) return gerr(CL_E_STATE, "the event trace is not available in the partitioned mode");
  if (g->go_seed) return gerr(CL_E_STATE, "the partitioned mode takes the counter hash or an explicit delay schedule");
  if (node_lo < 0 || node_lo > node_hi || node_hi > g->n || node_lo % kGThreads ||
      (node_hi != g->n && node_hi % kGThreads))
    return gerr(CL_E_INVALID, "node range [%d, %d) must be block-aligned (%d) within [0, %d)", node_lo, node_hi,
                kGThreads, g->n);
  if ((rc = g->ensure_device())) return rc;
  GHIP(hipSetDevice(g->device));
  bool realloc = false;
  if ((rc = g->ensure_state(&realloc)) || (rc = g->ensure_sched()) || (rc = g->upload_ops())) return rc;
  const size_t N = (size_t)g->n;
  if ((rc = g->d_outbox.ensure(N)) || (rc = g->d_out_n.ensure(4)) || (rc = g->d_rmlist.ensure(N)) ||
      (rc = g->d_reports.ensure(N)) || (rc = g->d_trigv.ensure(N)) || (rc = g->d_rdraw.ensure(N)) ||
      (rc = g->d_pop.ensure(1)))
    return rc;
  g->part = true;
  g->part_lo = node_lo;
  g->part_hi = node_hi;
  g->fill_params();
  if ((rc = g->k_err(cg_launch_reset(g->P, g->d_init_tok.p, g->stream)))) return rc;
  GHIP(hipMemsetAsync(g->d_trigv.p, 0, N * sizeof(int32_t), g->stream));
  GHIP(hipStreamSynchronize(g->stream));
  g->time = 0;
  g->hang = false;
  g->executed = g->prog.size();
  g->state_valid = true;
  return CL_OK;
}

int cl_graph_part_snapshot(cl_graph* g, int32_t node, int32_t* out_sid) {
  G_CHECK(g);
  G_PART(g);
  if (node < 0 || node >= g->n) return gerr(CL_E_UNKNOWN_NODE, "snapshot at unknown rank %d", node);
  if (g->n_sids >= g->s_cap) return gerr(CL_E_LIMIT, "more than %d snapshots (cl_graph_set_limits)", g->s_cap);
  const GOp op{GOP_SNAP, node, g->n_sids, 0};
  // stream-ordered: a k_hostops of an earlier call may still be queued on g->stream and read
  // d_pop (a null-stream hipMemcpy does not wait for the non-blocking stream: two snapshots
  // started back to back raced here)
  GHIP(hipMemcpyAsync(g->d_pop.p, &op, sizeof op, hipMemcpyHostToDevice, g->stream));
  GParams q = g->P;
  q.ops = g->d_pop.p;
  int rc = g->k_err(cg_launch_hostops(q, (int32_t)g->time, 0, 1, g->stream));
  if (rc) return rc;
  GHIP(hipStreamSynchronize(g->stream));  // (`op` is a stack copy)
  if (out_sid) *out_sid = g->n_sids;
  g->n_sids++;
  return CL_OK;
}

int cl_graph_part_pick(cl_graph* g, int32_t* rows, int64_t cap, int64_t* n_rows) {
  G_CHECK(g);
  G_PART(g);
  if (!n_rows || (cap > 0 && !rows)) return gerr(CL_E_INVALID, "null output");
  if (g->time + 1 > kMaxGraphTime) return gerr(CL_E_LIMIT, "simulated time would exceed %lld ticks", (long long)kMaxGraphTime);
  ++g->time;
  int rc = g->k_err(cg_launch_part_pick(g->P, (int32_t)g->time, g->stream));
  if (rc) return rc;
  uint32_t cnt[4];
  GHIP(hipMemcpyAsync(cnt, g->d_out_n.p, sizeof cnt, hipMemcpyDeviceToHost, g->stream));
  GHIP(hipStreamSynchronize(g->stream));
  *n_rows = cnt[0];
  if ((int64_t)cnt[0] > cap) return gerr(CL_E_LIMIT, "%u outgoing deliveries exceed cap %lld", cnt[0], (long long)cap);
  if (cnt[0]) GHIP(hipMemcpy(rows, g->d_outbox.p, cnt[0] * sizeof(PDel), hipMemcpyDeviceToHost));
  return CL_OK;
}

int cl_graph_part_receive(cl_graph* g, const int32_t* rows, int64_t n, int32_t* reports, int64_t cap,
                          int64_t* n_reports) {
  G_CHECK(g);
  G_PART(g);
  if (!n_reports || (n > 0 && !rows) || (cap > 0 && !reports)) return gerr(CL_E_INVALID, "null array");
  if (n < 0 || n > g->n) return gerr(CL_E_INVALID, "%lld incoming deliveries", (long long)n);
  int rc = g->d_inbox.ensure((size_t)n);
  if (rc) return rc;
  for (int64_t i = 0; i < n; ++i) {
    const int32_t* r = rows + 4 * i;
    if (r[1] < g->part_lo || r[1] >= g->part_hi || r[0] < 0 || r[0] >= g->n || r[2] < 0 || r[2] >= g->e)
      return gerr(CL_E_INVALID, "delivery %lld is not addressed to this device's nodes", (long long)i);
  }
  if (n) GHIP(hipMemcpyAsync(g->d_inbox.p, rows, (size_t)n * sizeof(PDel), hipMemcpyHostToDevice, g->stream));
  if ((rc = g->k_err(cg_launch_part_receive(g->P, (int32_t)g->time, g->d_inbox.p, (int32_t)n, g->stream)))) return rc;
  uint32_t cnt[4];
  GHIP(hipMemcpyAsync(cnt, g->d_out_n.p, sizeof cnt, hipMemcpyDeviceToHost, g->stream));
  GHIP(hipStreamSynchronize(g->stream));
  *n_reports = cnt[2];
  if ((int64_t)cnt[2] > cap) return gerr(CL_E_LIMIT, "%u reports exceed cap %lld", cnt[2], (long long)cap);
  if (cnt[2]) GHIP(hipMemcpy(reports, g->d_reports.p, cnt[2] * sizeof(int2), hipMemcpyDeviceToHost));
  return CL_OK;
}

int cl_graph_part_tally(cl_graph* g, int32_t step, const int32_t* reports, int64_t n, int64_t* totals) {
  G_CHECK(g);
  G_PART(g);
  if (!totals || (n > 0 && !reports)) return gerr(CL_E_INVALID, "null array");
  if (n < 0 || n > g->n) return gerr(CL_E_INVALID, "%lld reports", (long long)n);
  for (int64_t i = 0; i < n; ++i)
    if (reports[2 * i] < g->part_lo || reports[2 * i] >= g->part_hi || reports[2 * i + 1] < 0)
      return gerr(CL_E_INVALID, "report %lld is not about this device's senders", (long long)i);
  int rc = g->d_rep_in.ensure((size_t)n);
  if (rc) return rc;
  if (n) GHIP(hipMemcpyAsync(g->d_rep_in.p, reports, (size_t)n * sizeof(int2), hipMemcpyHostToDevice, g->stream));
  if ((rc = g->k_err(cg_launch_part_tally(g->P, step, g->d_rep_in.p, (int32_t)n, g->stream)))) return rc;
  GScal sc;
  GHIP(hipMemcpyAsync(&sc, g->d_sc.p, sizeof sc, hipMemcpyDeviceToHost, g->stream));
  GHIP(hipStreamSynchronize(g->stream));
  totals[0] = (int64_t)sc.tot_trig;
  totals[1] = (int64_t)sc.tot_send;
  totals[2] = sc.status;
  return CL_OK;
}

int cl_graph_part_freeze(cl_graph* g, int32_t status) {
  G_CHECK(g);
  G_PART(g);
  if (status <= 0) return gerr(CL_E_INVALID, "freeze needs a nonzero status");
  GScal sc;
  GHIP(hipMemcpyAsync(&sc, g->d_sc.p, sizeof sc, hipMemcpyDeviceToHost, g->stream));
  GHIP(hipStreamSynchronize(g->stream));
  if (sc.status) return CL_OK;
  GHIP(hipMemcpyAsync(&g->d_sc.p->status, &status, sizeof status, hipMemcpyHostToDevice, g->stream));
  GHIP(hipStreamSynchronize(g->stream));
  return CL_OK;
}

int cl_graph_part_bases(cl_graph* g, const int64_t* bases, const int32_t* s0, int64_t n, int64_t* draw0) {
  G_CHECK(g);
  G_PART(g);
  if (!bases || (n > 0 && (!s0 || !draw0))) return gerr(CL_E_INVALID, "null array");
  if (n < 0 || n > g->n) return gerr(CL_E_INVALID, "%lld reports", (long long)n);
  for (int64_t i = 0; i < n; ++i)
    if (s0[i] < g->part_lo || s0[i] >= g->part_hi) return gerr(CL_E_INVALID, "sender %d is not this device's", s0[i]);
  int rc;
  if ((rc = g->d_s0.ensure((size_t)n)) || (rc = g->d_draw0.ensure((size_t)n))) return rc;
  if (n) GHIP(hipMemcpyAsync(g->d_s0.p, s0, (size_t)n * sizeof(int32_t), hipMemcpyHostToDevice, g->stream));
  if ((rc = g->k_err(cg_launch_part_bases(g->P, bases[0], bases[1], bases[2], bases[3], g->d_s0.p, (int32_t)n,
                                          g->d_draw0.p, g->stream))))
    return rc;
  if (n) GHIP(hipMemcpyAsync(draw0, g->d_draw0.p, (size_t)n * sizeof(int64_t), hipMemcpyDeviceToHost, g->stream));
  GHIP(hipStreamSynchronize(g->stream));
  return CL_OK;
}

int cl_graph_part_push(cl_graph* g, int32_t step, const int64_t* replies, int64_t n) {
  G_CHECK(g);
  G_PART(g);
  if (n > 0 && !replies) return gerr(CL_E_INVALID, "null array");
  if (n < 0 || n > g->n) return gerr(CL_E_INVALID, "%lld replies", (long long)n);
  for (int64_t i = 0; i < n; ++i)
    if (replies[2 * i] < 0 || replies[2 * i] >= g->n || (replies[2 * i] >= g->part_lo && replies[2 * i] < g->part_hi))
      return gerr(CL_E_INVALID, "reply %lld names sender %lld", (long long)i, (long long)replies[2 * i]);
  int rc = g->d_replies.ensure(2 * (size_t)n);
  if (rc) return rc;
  if (n) GHIP(hipMemcpyAsync(g->d_replies.p, replies, 2 * (size_t)n * sizeof(int64_t), hipMemcpyHostToDevice, g->stream));
  if ((rc = g->k_err(cg_launch_part_push(g->P, (int32_t)g->time, step, g->d_replies.p, (int32_t)n, g->stream)))) return rc;
  GHIP(hipStreamSynchronize(g->stream));  // (the staged rows must outlive the launch)
  return CL_OK;
}

// ---- partitioned mode, device-resident exchange (clgraph.h cl_graph_part_dev_*) ----------
int cl_graph_set_stream(cl_graph* g, void* stream) {
  G_CHECK(g);
  int rc = g->ensure_device();
  if (rc) return rc;
  GHIP(hipSetDevice(g->device));
  GHIP(hipStreamSynchronize(g->stream));
  g->stream = stream ? (hipStream_t)stream : g->own_stream;
  return CL_OK;
}

#define G_DEV(g)                                                                                  \
  do {                                                                                            \
    G_CHECK(g);                                                                                   \
    G_PART(g);                                                                                    \
    if (!(g)->bk_send) return gerr(CL_E_STATE, "no device exchange buffers (cl_graph_part_dev_bind)"); \
  } while (0)

int cl_graph_part_dev_bind(cl_graph* g, int32_t world, int32_t rank, int32_t span, int64_t cap, void* send,
                           void* recv, void* tot_send, void* tot_recv) {
  G_CHECK(g);
  G_PART(g);
  if (world < 1 || rank < 0 || rank >= world || span <= 0 || span % kGThreads)
    return gerr(CL_E_INVALID, "rank %d of %d, span %d (a positive multiple of %d)", rank, world, span, kGThreads);
  if (g->part_lo != rank * span || g->part_hi != std::min<int64_t>((int64_t)(rank + 1) * span, g->n))
    return gerr(CL_E_INVALID, "rank %d x span %d is not this device's range [%d, %d)", rank, span, g->part_lo,
                g->part_hi);
  if ((int64_t)world * span < g->n) return gerr(CL_E_INVALID, "%d ranks x %d nodes do not cover %d", world, span, g->n);
  if (cap < 1 || cap > g->n) return gerr(CL_E_INVALID, "bucket capacity %lld", (long long)cap);
  if (!send || !recv || !tot_send || !tot_recv) return gerr(CL_E_INVALID, "null exchange buffer");
  GHIP(hipSetDevice(g->device));
  int rc = g->d_bk_cnt.ensure((size_t)world);
  if (rc) return rc;
  GHIP(hipMemsetAsync(g->d_bk_cnt.p, 0, (size_t)world * sizeof(uint32_t), g->stream));
  GHIP(hipStreamSynchronize(g->stream));
  g->bk_world = world;
  g->bk_rank = rank;
  g->bk_span = span;
  g->bk_cap = (int32_t)cap;
  g->bk_send = send;
  g->bk_recv = recv;
  g->tot_send = tot_send;
  g->tot_recv = tot_recv;
  g->fill_params();
  return CL_OK;
}

int cl_graph_part_dev_seal(cl_graph* g) {
  G_DEV(g);
  return g->k_err(cg_launch_part_dev_seal(g->P, g->stream));
}

int cl_graph_part_dev_pick(cl_graph* g) {
  G_DEV(g);
  if (g->time + 1 > kMaxGraphTime) return gerr(CL_E_LIMIT, "simulated time would exceed %lld ticks", (long long)kMaxGraphTime);
  ++g->time;
  return g->k_err(cg_launch_part_dev_pick(g->P, (int32_t)g->time, g->stream));
}

int cl_graph_part_dev_receive(cl_graph* g) {
  G_DEV(g);
  return g->k_err(cg_launch_part_dev_receive(g->P, (int32_t)g->time, g->stream));
}

int cl_graph_part_dev_tally(cl_graph* g, int32_t step) {
  G_DEV(g);
  return g->k_err(cg_launch_part_dev_tally(g->P, step, g->stream));
}

int cl_graph_part_dev_bases(cl_graph* g) {
  G_DEV(g);
  return g->k_err(cg_launch_part_dev_bases(g->P, g->stream));
}

int cl_graph_part_dev_push(cl_graph* g, int32_t step) {
  G_DEV(g);
  return g->k_err(cg_launch_part_dev_push(g->P, (int32_t)g->time, step, g->stream));
}

}  // extern "C"
