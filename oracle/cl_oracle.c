/*
 * cl_oracle.c -- CPU restatement of the reference Chandy-Lamport simulator.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker: it may be loaded by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the
 * product path (chandy-lamport-distributed-snapshot-algorithm_amd/).  It restates
 * the reference literally -- string node IDs, lexicographic iteration, per-snapshot
 * per-link recording flags and recorded message lists, unbounded FIFOs -- so that it
 * shares no data layout or shortcut with the GPU engine it checks.
 *
 * Parity pin: the reference is Go and no Go toolchain exists in this image, so it
 * cannot be built (oracle/_ref is empty).  The restatement is pinned instead by the
 * reference's own golden vectors: all 21 test_data .snap snapshots of the 7 tests in
 * snapshot_test.go:46-108, reproduced under the Go math/rand stream for seed
 * 8053172852482175523+1 (snapshot_test.go:9,20), which is restated below and pinned
 * by Go's published math/rand known answers (tests/golden/go_rng_kat.json).
 *
 * Reference map (paths relative to /root/reference/chandy_lamport):
 *   go_rng_*            Go stdlib math/rand rngSource / Int31n (Go 1.22, go.mod:3)
 *   orc_add_node        sim.go:40-43, node.go:45-55
 *   orc_add_link        sim.go:46-56, node.go:87-94
 *   orc_tick            sim.go:71-95
 *   get_receive_time    sim.go:100-102
 *   orc_start_snapshot  sim.go:105-123, node.go:198-212
 *   notify_completed    sim.go:126-131
 *   orc_collect         sim.go:134-173
 *   create_local        node.go:58-84
 *   send_to_neighbors   node.go:97-109
 *   orc_send_tokens     node.go:112-131
 *   handle_packet       node.go:140-185 (HandleMarker :149-171, HandleToken :174-185)
 *   finalize            node.go:188-195
 *   queue ops           queue.go:14-28 (push front / pop back == FIFO)
 *   orc_read_topology   test_common.go:29-68
 *   orc_read_events     test_common.go:79-140 (incl. the inverted comment test :90)
 * Every reference log.Fatal* becomes a per-simulator status; the simulator then freezes.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "go_rng_cooked.h"

/* ------------------------------------------------------------------------- */
/* Go math/rand (rng.go, rand.go) restatement                                 */
/* ------------------------------------------------------------------------- */
#define GO_LEN 607
#define GO_TAP 273
#define GO_I32MAX 2147483647LL

typedef struct {
    int tap, feed;
    int64_t vec[GO_LEN];
} go_rng;

static int32_t go_seedrand(int32_t x) {
    const int32_t A = 48271, Q = 44488, R = 3399;
    int32_t hi = x / Q, lo = x % Q;
    x = A * lo - R * hi;
    if (x < 0) x += (int32_t)GO_I32MAX;
    return x;
}

static void go_rng_seed(go_rng* r, int64_t seed) {
    r->tap = 0;
    r->feed = GO_LEN - GO_TAP;
    seed = seed % GO_I32MAX;
    if (seed < 0) seed += GO_I32MAX;
    if (seed == 0) seed = 89482311;
    int32_t x = (int32_t)seed;
    for (int i = -20; i < GO_LEN; i++) {
        x = go_seedrand(x);
        if (i >= 0) {
            uint64_t u = (uint64_t)(int64_t)x << 40;
            x = go_seedrand(x);
            u ^= (uint64_t)(int64_t)x << 20;
            x = go_seedrand(x);
            u ^= (uint64_t)(int64_t)x;
            u ^= (uint64_t)ORC_RNG_COOKED[i];
            r->vec[i] = (int64_t)u;
        }
    }
}

static uint64_t go_rng_uint64(go_rng* r) {
    if (--r->tap < 0) r->tap += GO_LEN;
    if (--r->feed < 0) r->feed += GO_LEN;
    uint64_t x = (uint64_t)r->vec[r->feed] + (uint64_t)r->vec[r->tap];
    r->vec[r->feed] = (int64_t)x;
    return x;
}

static int64_t go_int63(go_rng* r) { return (int64_t)(go_rng_uint64(r) & 0x7fffffffffffffffULL); }
static int32_t go_int31(go_rng* r) { return (int32_t)(go_int63(r) >> 32); }

static int32_t go_int31n(go_rng* r, int32_t n) {
    if ((n & (n - 1)) == 0) return go_int31(r) & (n - 1);
    int32_t max = (int32_t)((1LL << 31) - 1 - (int64_t)((1ULL << 31) % (uint32_t)n));
    int32_t v = go_int31(r);
    while (v > max) v = go_int31(r);
    return v % n;
}

/* rand.Intn for 0 < n <= 1<<31-1 (rand.go: Intn -> Int31n) */
static int go_intn(go_rng* r, int n) { return (int)go_int31n(r, (int32_t)n); }

void orc_go_int63_seq(int64_t seed, int64_t n, int64_t* out) {
    go_rng r;
    go_rng_seed(&r, seed);
    for (int64_t i = 0; i < n; i++) out[i] = go_int63(&r);
}

void orc_go_intn_seq(int64_t seed, int32_t bound, int64_t n, int32_t* out) {
    go_rng r;
    go_rng_seed(&r, seed);
    for (int64_t i = 0; i < n; i++) out[i] = go_intn(&r, bound);
}

/* ------------------------------------------------------------------------- */
/* Simulator state (common.go, node.go, sim.go, queue.go)                     */
/* ------------------------------------------------------------------------- */
enum {
    ORC_OK = 0,
    ORC_FATAL_INSUFFICIENT_TOKENS = 1, /* node.go:113-116 */
    ORC_FATAL_UNKNOWN_DEST = 2,        /* node.go:121-124 */
    ORC_HANG = 4,                      /* drain never ends (test_common.go:124-132) */
    ORC_DELAY_EXHAUSTED = 5,           /* replayed schedule shorter than the run */
    ORC_ERR_API = -1,                  /* unknown node etc.: log.Fatalf / nil deref */
    ORC_ERR_PARSE = -2,
};

#define MAX_DELAY 5 /* sim.go:10 */

typedef struct {
    int is_marker; /* common.go:28-31 */
    int64_t data;
} orc_msg;

typedef struct {
    int src, dest; /* node indices (stable, insertion order) */
    orc_msg msg;
    int64_t receive_time; /* common.go:43-50 */
} orc_event;

typedef struct { /* queue.go: list with PushFront / Remove(Back) == FIFO */
    orc_event* buf;
    int64_t head, len, cap;
} orc_queue;

typedef struct {
    int src, dest;
    orc_queue q;
} orc_link;

typedef struct {
    int64_t* v;
    int64_t n, cap;
} i64vec;

typedef struct { /* node.go:34-43 LocalSnapshot */
    int exists;
    int64_t num_tokens_in_node;
    unsigned char* is_link_recording; /* indexed like node.in_links */
    int64_t num_links_being_recorded;
    i64vec* incoming; /* incomingMessages[src], indexed like node.in_links */
    int finalized;
} orc_local;

typedef struct {
    char* id;
    int64_t tokens;
    int* out_links; /* link indices */
    int n_out, cap_out;
    int* in_links;
    int n_in, cap_in;
    orc_local* snaps; /* activeSnapshots[sid] */
    int n_snaps;
} orc_node;

typedef struct {
    int64_t push, peek, pop_tok, pop_mk, recorded, draws, completed;
} orc_counters;

/* logger.go:18-23 LogEvent, with node IDs as sort ranks: {epoch, kind, node, other,
 * data, nodeTokens}; kinds as CL_LOG_* in include/clsnap.h */
enum { LOG_SENT_TOKEN = 0, LOG_SENT_MARKER, LOG_RECV_TOKEN, LOG_RECV_MARKER, LOG_START, LOG_END };
typedef struct {
    int64_t epoch;
    int32_t kind, node, other;
    int64_t data, tokens;
} orc_log_rec;

typedef struct orc_sim {
    int64_t time;              /* sim.go:13 */
    int next_snapshot_id;      /* sim.go:14 */
    orc_node* nodes;
    int n_nodes, cap_nodes;
    orc_link* links;
    int n_links, cap_links;
    int* sorted;               /* getSortedKeys(sim.nodes), common.go:135-146 */
    int* completed_count;      /* activeSnapshotsWG[sid] as a countdown of N */
    int* collected;            /* drain bookkeeping (test_common.go:124-132) */
    int64_t* completion_tick;
    int cap_sids;
    int status;
    /* delay source */
    int use_go;
    int use_hash;              /* counter-hash delays (synthetic workloads) */
    uint64_t hash_seed;
    go_rng rng;
    const uint8_t* sched;
    int64_t sched_len, sched_pos;
    orc_counters cnt;
    int64_t drain_ticks;
    /* Logger (logger.go:12-76): epoch = time (NewEpoch per Tick, sim.go:73) */
    int log_on;
    orc_log_rec* log;
    int64_t n_log, cap_log;
} orc_sim;

static void* xrealloc(void* p, size_t n) {
    void* q = realloc(p, n ? n : 1);
    if (!q) { fprintf(stderr, "oracle: out of memory\n"); abort(); }
    return q;
}

orc_sim* orc_new(void) {
    orc_sim* s = (orc_sim*)calloc(1, sizeof(orc_sim));
    go_rng_seed(&s->rng, 1); /* Go's default source before rand.Seed */
    s->use_go = 1;
    return s;
}

static void queue_free(orc_queue* q) { free(q->buf); memset(q, 0, sizeof(*q)); }

void orc_free(orc_sim* s) {
    if (!s) return;
    for (int i = 0; i < s->n_nodes; i++) {
        orc_node* n = &s->nodes[i];
        for (int k = 0; k < n->n_snaps; k++) {
            orc_local* l = &n->snaps[k];
            if (!l->exists) continue;
            free(l->is_link_recording);
            for (int j = 0; j < n->n_in; j++) free(l->incoming[j].v);
            free(l->incoming);
        }
        free(n->snaps);
        free(n->out_links);
        free(n->in_links);
        free(n->id);
    }
    for (int i = 0; i < s->n_links; i++) queue_free(&s->links[i].q);
    free(s->nodes); free(s->links); free(s->sorted);
    free(s->completed_count); free(s->collected); free(s->completion_tick);
    free(s->log);
    free(s);
}

void orc_seed_go(orc_sim* s, int64_t seed) { s->use_go = 1; s->use_hash = 0; go_rng_seed(&s->rng, seed); }

/* ------------------------------------------------------------------------- */
/* Counter hash for the synthetic workloads.  Same     */
/* definition as the engine's cg_hash (csrc/cg_engine.h), restated here so the */
/* two are checked against each other rather than shared.                      */
/* ------------------------------------------------------------------------- */
static uint64_t mix64(uint64_t z);

uint64_t orc_counter_hash(uint64_t seed, uint64_t a, uint64_t b) {
    uint64_t h = mix64(seed ^ (a * 0x9E3779B97F4A7C15ULL));
    return mix64(h ^ (b * 0xD6E8FEB86659FD93ULL));
}

/* Delay of draw k under the counter-hash source: replaces rand.Intn(maxDelay) at
 * sim.go:101 by a pure function of the instance's draw index, so the reference's
 * draw ORDER (host events in order, then deliveries in sender order) still decides
 * every delay. */
int orc_counter_delay(uint64_t seed, uint64_t k) {
    return (int)((orc_counter_hash(seed, k, 0) >> 32) % 5u);
}

void orc_use_counter_hash(orc_sim* s, uint64_t seed) {
    s->use_go = 0; s->use_hash = 1; s->hash_seed = seed;
}

/* Replay a per-message delay schedule (values in [0, MAX_DELAY)). The caller keeps
 * the buffer alive. This replaces rand.Intn(maxDelay) at sim.go:101. */
void orc_use_schedule(orc_sim* s, const uint8_t* delays, int64_t len) {
    s->use_go = 0; s->use_hash = 0; s->sched = delays; s->sched_len = len; s->sched_pos = 0;
}

int orc_status(const orc_sim* s) { return s->status; }
int64_t orc_time(const orc_sim* s) { return s->time; }
int orc_num_nodes(const orc_sim* s) { return s->n_nodes; }
int orc_num_snapshots(const orc_sim* s) { return s->next_snapshot_id; }
void orc_counters_get(const orc_sim* s, int64_t* out7) {
    out7[0] = s->cnt.push; out7[1] = s->cnt.peek; out7[2] = s->cnt.pop_tok;
    out7[3] = s->cnt.pop_mk; out7[4] = s->cnt.recorded; out7[5] = s->cnt.draws;
    out7[6] = s->cnt.completed;
}

static int find_node(const orc_sim* s, const char* id) {
    for (int i = 0; i < s->n_nodes; i++)
        if (strcmp(s->nodes[i].id, id) == 0) return i;
    return -1;
}

static const orc_sim* g_sort_sim;
static int cmp_node_ids(const void* a, const void* b) {
    return strcmp(g_sort_sim->nodes[*(const int*)a].id, g_sort_sim->nodes[*(const int*)b].id);
}

static void resort(orc_sim* s) { /* getSortedKeys over sim.nodes (sort.Strings) */
    s->sorted = (int*)xrealloc(s->sorted, sizeof(int) * (size_t)s->n_nodes);
    for (int i = 0; i < s->n_nodes; i++) s->sorted[i] = i;
    /* qsort comparator needs the sim; single-threaded per sim during topology build */
    static pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
    pthread_mutex_lock(&mu);
    g_sort_sim = s;
    qsort(s->sorted, (size_t)s->n_nodes, sizeof(int), cmp_node_ids);
    pthread_mutex_unlock(&mu);
}

/* sim.go:40-43 AddNode */
int orc_add_node(orc_sim* s, const char* id, int64_t tokens) {
    if (find_node(s, id) >= 0) return ORC_ERR_API; /* replacing a wired node is ill-defined */
    if (s->n_nodes == s->cap_nodes) {
        s->cap_nodes = s->cap_nodes ? 2 * s->cap_nodes : 16;
        s->nodes = (orc_node*)xrealloc(s->nodes, sizeof(orc_node) * (size_t)s->cap_nodes);
    }
    orc_node* n = &s->nodes[s->n_nodes++];
    memset(n, 0, sizeof(*n));
    n->id = strdup(id);
    n->tokens = tokens;
    resort(s);
    return ORC_OK;
}

/* order a node's out links by dest id, in links by src id (getSortedKeys) */
static void insert_sorted(orc_sim* s, int** arr, int* n, int* cap, int link, int by_dest) {
    if (*n == *cap) {
        *cap = *cap ? 2 * *cap : 4;
        *arr = (int*)xrealloc(*arr, sizeof(int) * (size_t)*cap);
    }
    const char* key = s->nodes[by_dest ? s->links[link].dest : s->links[link].src].id;
    int pos = *n;
    while (pos > 0) {
        const orc_link* o = &s->links[(*arr)[pos - 1]];
        const char* ok = s->nodes[by_dest ? o->dest : o->src].id;
        if (strcmp(ok, key) <= 0) break;
        (*arr)[pos] = (*arr)[pos - 1];
        pos--;
    }
    (*arr)[pos] = link;
    (*n)++;
}

/* sim.go:46-56 AddLink -> node.go:87-94 AddOutboundLink */
int orc_add_link(orc_sim* s, const char* src, const char* dest) {
    int a = find_node(s, src), b = find_node(s, dest);
    if (a < 0 || b < 0) return ORC_ERR_API; /* log.Fatalf("Node %v does not exist") */
    if (a == b) return ORC_OK;              /* node.go:88-90 */
    orc_node* na = &s->nodes[a];
    for (int k = 0; k < na->n_out; k++) {
        orc_link* l = &s->links[na->out_links[k]];
        if (l->dest == b) { /* map assignment replaces the link: fresh queue */
            queue_free(&l->q);
            return ORC_OK;
        }
    }
    if (s->n_links == s->cap_links) {
        s->cap_links = s->cap_links ? 2 * s->cap_links : 16;
        s->links = (orc_link*)xrealloc(s->links, sizeof(orc_link) * (size_t)s->cap_links);
    }
    int li = s->n_links++;
    memset(&s->links[li], 0, sizeof(orc_link));
    s->links[li].src = a;
    s->links[li].dest = b;
    insert_sorted(s, &na->out_links, &na->n_out, &na->cap_out, li, 1);
    orc_node* nb = &s->nodes[b];
    insert_sorted(s, &nb->in_links, &nb->n_in, &nb->cap_in, li, 0);
    return ORC_OK;
}

static void queue_push(orc_queue* q, orc_event e) {
    if (q->len == q->cap) {
        int64_t nc = q->cap ? 2 * q->cap : 8;
        orc_event* nb = (orc_event*)xrealloc(NULL, sizeof(orc_event) * (size_t)nc);
        for (int64_t i = 0; i < q->len; i++) nb[i] = q->buf[(q->head + i) % q->cap];
        free(q->buf);
        q->buf = nb; q->cap = nc; q->head = 0;
    }
    q->buf[(q->head + q->len) % q->cap] = e;
    q->len++;
}

static orc_event* queue_peek(orc_queue* q) { return &q->buf[q->head]; }

static orc_event queue_pop(orc_queue* q) {
    orc_event e = q->buf[q->head];
    q->head = (q->head + 1) % q->cap;
    q->len--;
    return e;
}

/* sim.go:100-102 GetReceiveTime */
static int get_receive_time(orc_sim* s, int64_t* rt) {
    int d;
    if (s->use_go) {
        d = go_intn(&s->rng, MAX_DELAY);
    } else if (s->use_hash) {
        d = orc_counter_delay(s->hash_seed, (uint64_t)s->cnt.draws);
    } else {
        if (s->sched_pos >= s->sched_len) return ORC_DELAY_EXHAUSTED;
        d = s->sched[s->sched_pos++];
    }
    s->cnt.draws++;
    *rt = s->time + 1 + d;
    return ORC_OK;
}

static void ensure_sids(orc_sim* s, int sid) {
    if (sid < s->cap_sids) return;
    int nc = s->cap_sids ? s->cap_sids : 8;
    while (nc <= sid) nc *= 2;
    s->completed_count = (int*)xrealloc(s->completed_count, sizeof(int) * (size_t)nc);
    s->collected = (int*)xrealloc(s->collected, sizeof(int) * (size_t)nc);
    s->completion_tick = (int64_t*)xrealloc(s->completion_tick, sizeof(int64_t) * (size_t)nc);
    for (int i = s->cap_sids; i < nc; i++) {
        s->completed_count[i] = 0; s->collected[i] = 0; s->completion_tick[i] = -1;
    }
    s->cap_sids = nc;
}

static orc_local* local_snap(orc_node* n, int sid) {
    if (sid >= n->n_snaps) return NULL;
    return n->snaps[sid].exists ? &n->snaps[sid] : NULL;
}

/* node.go:58-84 CreateLocalSnapshot; src_in = index into in_links or -1 for "" */
static int rank_of(const orc_sim* s, int node) {
    for (int a = 0; a < s->n_nodes; a++)
        if (s->sorted[a] == node) return a;
    return -1;
}

/* Logger.RecordEvent (logger.go:71-76): node's tokens at the time of the event */
static void log_event(orc_sim* s, int kind, int node, int other, int64_t data) {
    if (!s->log_on) return;
    if (s->n_log == s->cap_log) {
        s->cap_log = s->cap_log ? 2 * s->cap_log : 256;
        s->log = (orc_log_rec*)xrealloc(s->log, sizeof(orc_log_rec) * (size_t)s->cap_log);
    }
    orc_log_rec* r = &s->log[s->n_log++];
    r->epoch = s->time;
    r->kind = kind;
    r->node = rank_of(s, node);
    r->other = other >= 0 ? rank_of(s, other) : -1;
    r->data = data;
    r->tokens = s->nodes[node].tokens;
}

void orc_log_enable(orc_sim* s, int on) { s->log_on = on; }
int64_t orc_log_count(const orc_sim* s) { return s->n_log; }
void orc_log_get(const orc_sim* s, int64_t* out /* [n_log][6] */) {
    for (int64_t i = 0; i < s->n_log; i++) {
        const orc_log_rec* r = &s->log[i];
        int64_t* o = out + 6 * i;
        o[0] = r->epoch; o[1] = r->kind; o[2] = r->node; o[3] = r->other; o[4] = r->data; o[5] = r->tokens;
    }
}

static void create_local(orc_sim* s, int node, int sid, int src_in) {
    orc_node* n = &s->nodes[node];
    (void)s;
    if (sid >= n->n_snaps) {
        n->snaps = (orc_local*)xrealloc(n->snaps, sizeof(orc_local) * (size_t)(sid + 1));
        for (int k = n->n_snaps; k <= sid; k++) memset(&n->snaps[k], 0, sizeof(orc_local));
        n->n_snaps = sid + 1;
    }
    orc_local* l = &n->snaps[sid];
    l->exists = 1;
    l->num_tokens_in_node = n->tokens;
    l->is_link_recording = (unsigned char*)xrealloc(NULL, (size_t)n->n_in);
    l->incoming = (i64vec*)calloc((size_t)(n->n_in ? n->n_in : 1), sizeof(i64vec));
    for (int j = 0; j < n->n_in; j++) l->is_link_recording[j] = 1;
    l->num_links_being_recorded = n->n_in;
    if (src_in >= 0) {
        l->is_link_recording[src_in] = 0;
        l->num_links_being_recorded = n->n_in - 1;
    }
    l->finalized = 0;
}

/* node.go:97-109 SendToNeighbors: one draw per out link, dest-sorted */
static int send_to_neighbors(orc_sim* s, int node, orc_msg m) {
    orc_node* n = &s->nodes[node];
    for (int k = 0; k < n->n_out; k++) {
        orc_link* l = &s->links[n->out_links[k]];
        log_event(s, m.is_marker ? LOG_SENT_MARKER : LOG_SENT_TOKEN, node, l->dest, m.data); /* node.go:100 */
        orc_event e;
        e.src = l->src; e.dest = l->dest; e.msg = m;
        int rc = get_receive_time(s, &e.receive_time);
        if (rc) return rc;
        queue_push(&l->q, e);
        s->cnt.push++;
    }
    return ORC_OK;
}

/* node.go:198-212 Node.StartSnapshot */
static int node_start_snapshot(orc_sim* s, int node, int sid) {
    if (!local_snap(&s->nodes[node], sid)) create_local(s, node, sid, -1);
    orc_msg m = {1, sid};
    return send_to_neighbors(s, node, m);
}

/* sim.go:126-131 NotifyCompletedSnapshot */
static void notify_completed(orc_sim* s, int node, int sid) {
    log_event(s, LOG_END, node, -1, sid); /* sim.go:127 */
    s->completed_count[sid]++;
    if (s->completed_count[sid] == s->n_nodes) {
        s->completion_tick[sid] = s->time;
        s->cnt.completed++;
    }
}

static int in_index(const orc_sim* s, int node, int src) {
    const orc_node* n = &s->nodes[node];
    for (int j = 0; j < n->n_in; j++)
        if (s->links[n->in_links[j]].src == src) return j;
    return -1;
}

/* node.go:140-185 HandlePacket / HandleMarker / HandleToken */
static int handle_packet(orc_sim* s, int node, int src, orc_msg m) {
    orc_node* n = &s->nodes[node];
    int j = in_index(s, node, src);
    if (m.is_marker) {
        int sid = (int)m.data;
        if (!local_snap(n, sid)) {
            create_local(s, node, sid, j);
            int rc = node_start_snapshot(s, node, sid);
            if (rc) return rc;
            n = &s->nodes[node];
        } else {
            orc_local* l = local_snap(n, sid);
            l->is_link_recording[j] = 0;
            l->num_links_being_recorded--;
        }
        orc_local* l = local_snap(n, sid);
        if (l->num_links_being_recorded == 0) {
            l->finalized = 1; /* finalizeSnapshot: flattening happens at collect time */
            notify_completed(s, node, sid);
        }
    } else {
        n->tokens += m.data;
        for (int sid = 0; sid < n->n_snaps; sid++) { /* range node.activeSnapshots */
            orc_local* l = local_snap(n, sid);
            if (l && l->is_link_recording[j]) {
                i64vec* v = &l->incoming[j];
                if (v->n == v->cap) {
                    v->cap = v->cap ? 2 * v->cap : 4;
                    v->v = (int64_t*)xrealloc(v->v, sizeof(int64_t) * (size_t)v->cap);
                }
                v->v[v->n++] = m.data;
                s->cnt.recorded++;
            }
        }
    }
    return ORC_OK;
}

/* sim.go:71-95 Tick */
int orc_tick(orc_sim* s) {
    if (s->status) return s->status;
    s->time++;
    for (int a = 0; a < s->n_nodes; a++) {
        orc_node* n = &s->nodes[s->sorted[a]];
        for (int k = 0; k < n->n_out; k++) {
            orc_link* l = &s->links[n->out_links[k]];
            if (l->q.len > 0) {
                s->cnt.peek++;
                orc_event* e = queue_peek(&l->q);
                if (e->receive_time <= s->time) {
                    orc_event ev = queue_pop(&l->q);
                    if (ev.msg.is_marker) s->cnt.pop_mk++; else s->cnt.pop_tok++;
                    log_event(s, ev.msg.is_marker ? LOG_RECV_MARKER : LOG_RECV_TOKEN, ev.dest, ev.src,
                              ev.msg.data); /* sim.go:86 */
                    int rc = handle_packet(s, ev.dest, ev.src, ev.msg);
                    if (rc) { s->status = rc; return rc; }
                    break;
                }
            }
        }
    }
    return ORC_OK;
}

/* node.go:112-131 SendTokens (via sim.go:58-62 ProcessEvent); a, b node indices */
static int send_tokens_idx(orc_sim* s, int a, int b, int64_t num) {
    orc_node* n = &s->nodes[a];
    if (n->tokens < num) { s->status = ORC_FATAL_INSUFFICIENT_TOKENS; return s->status; }
    orc_link* l = NULL;
    for (int k = 0; k < n->n_out && b >= 0; k++)
        if (s->links[n->out_links[k]].dest == b) l = &s->links[n->out_links[k]];
    /* node.go:118: logged before the link check; the record's dest is -1 without a link */
    log_event(s, LOG_SENT_TOKEN, a, l ? b : -1, num);
    n->tokens -= num;
    if (!l) { s->status = ORC_FATAL_UNKNOWN_DEST; return s->status; }
    orc_event e;
    e.src = a; e.dest = b; e.msg.is_marker = 0; e.msg.data = num;
    int rc = get_receive_time(s, &e.receive_time);
    if (rc) { s->status = rc; return rc; }
    queue_push(&l->q, e);
    s->cnt.push++;
    return ORC_OK;
}

int orc_send_tokens(orc_sim* s, const char* src, const char* dest, int64_t num) {
    if (s->status) return s->status;
    int a = find_node(s, src);
    if (a < 0) return ORC_ERR_API; /* nil *Node dereference in the reference */
    return send_tokens_idx(s, a, find_node(s, dest), num);
}

/* sim.go:105-123 StartSnapshot on node index a */
static int start_snapshot_idx(orc_sim* s, int a, int* out_sid) {
    int sid = s->next_snapshot_id++;
    ensure_sids(s, sid);
    if (out_sid) *out_sid = sid;
    log_event(s, LOG_START, a, -1, sid); /* sim.go:109 */
    int rc = node_start_snapshot(s, a, sid);
    if (rc) s->status = rc;
    return rc;
}

/* sim.go:105-123 StartSnapshot */
int orc_start_snapshot(orc_sim* s, const char* node, int* out_sid) {
    if (s->status) return s->status;
    int a = find_node(s, node);
    if (a < 0) return ORC_ERR_API;
    int sid = s->next_snapshot_id++;
    ensure_sids(s, sid);
    if (out_sid) *out_sid = sid;
    log_event(s, LOG_START, a, -1, sid); /* sim.go:109 */
    int rc = node_start_snapshot(s, a, sid);
    if (rc) s->status = rc;
    return rc;
}

int orc_snapshot_complete(const orc_sim* s, int sid) {
    return sid < s->next_snapshot_id && s->completed_count[sid] == s->n_nodes;
}

int64_t orc_completion_tick(const orc_sim* s, int sid) {
    return sid < s->next_snapshot_id ? s->completion_tick[sid] : -1;
}

/* node tokens in sorted order (checkTokens, test_common.go:298-302) */
void orc_node_tokens(const orc_sim* s, int64_t* out) {
    for (int a = 0; a < s->n_nodes; a++) out[a] = s->nodes[s->sorted[a]].tokens;
}

const char* orc_node_id(const orc_sim* s, int sorted_index) {
    return s->nodes[s->sorted[sorted_index]].id;
}

/* sim.go:134-173 CollectSnapshot for a completed snapshot.
 * tokens[N] in sorted node order; messages as (src, dest) sorted-node ranks + amount,
 * per destination in sorted order, per source (in-link order), in recording order.
 * Returns the number of messages (may exceed cap: then only cap are written). */
int64_t orc_collect(const orc_sim* s, int sid, int64_t* tokens, int32_t* msg_src,
                    int32_t* msg_dest, int64_t* msg_amt, int64_t cap) {
    if (!orc_snapshot_complete(s, sid)) return -1;
    int* rank = (int*)xrealloc(NULL, sizeof(int) * (size_t)s->n_nodes);
    for (int a = 0; a < s->n_nodes; a++) rank[s->sorted[a]] = a;
    int64_t m = 0;
    for (int a = 0; a < s->n_nodes; a++) {
        const orc_node* n = &s->nodes[s->sorted[a]];
        const orc_local* l = &n->snaps[sid];
        tokens[a] = l->num_tokens_in_node;
        for (int j = 0; j < n->n_in; j++) {
            const i64vec* v = &l->incoming[j];
            for (int64_t k = 0; k < v->n; k++, m++) {
                if (m < cap) {
                    msg_src[m] = rank[s->links[n->in_links[j]].src];
                    msg_dest[m] = a;
                    msg_amt[m] = v->v[k];
                }
            }
        }
    }
    free(rank);
    return m;
}

/* ------------------------------------------------------------------------- */
/* Snapshot content hash (shared definition with the GPU engine) */
/* ------------------------------------------------------------------------- */
static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

/* Channels are ordered by (src id, dest id) lexicographically; nodes by id. */
uint64_t orc_snapshot_hash(const orc_sim* s, int sid) {
    if (!orc_snapshot_complete(s, sid)) return 0;
    uint64_t h = 0x9E3779B97F4A7C15ULL ^ (uint64_t)sid;
    for (int a = 0; a < s->n_nodes; a++)
        h = mix64(h ^ (uint64_t)s->nodes[s->sorted[a]].snaps[sid].num_tokens_in_node);
    uint64_t ch = 0;
    for (int a = 0; a < s->n_nodes; a++) {
        const orc_node* src = &s->nodes[s->sorted[a]];
        for (int k = 0; k < src->n_out; k++, ch++) {
            const orc_link* l = &s->links[src->out_links[k]];
            const orc_node* dn = &s->nodes[l->dest];
            int j = in_index(s, l->dest, l->src);
            const i64vec* v = &dn->snaps[sid].incoming[j];
            h = mix64(h ^ (ch << 32) ^ (uint64_t)v->n);
            for (int64_t q = 0; q < v->n; q++) h = mix64(h ^ (uint64_t)v->v[q]);
        }
    }
    return h;
}

/* ------------------------------------------------------------------------- */
/* Drivers: .top / .events (test_common.go:29-140)                            */
/* ------------------------------------------------------------------------- */
static char* read_file(const char* path, size_t* len) {
    FILE* f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    char* b = (char*)xrealloc(NULL, (size_t)n + 1);
    size_t got = fread(b, 1, (size_t)n, f);
    fclose(f);
    b[got] = 0;
    if (len) *len = got;
    return b;
}

static int is_go_space(char c) {
    return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r';
}

/* strings.Fields (ASCII whitespace) into at most maxf fields; returns count */
static int go_fields(char* line, char** f, int maxf) {
    int n = 0;
    char* p = line;
    while (*p) {
        while (*p && is_go_space(*p)) p++;
        if (!*p) break;
        char* st = p;
        while (*p && !is_go_space(*p)) p++;
        if (n < maxf) f[n] = st;
        n++;
        if (*p) *p++ = 0;
    }
    return n;
}

/* strconv.Atoi: optional sign then decimal digits only */
static int go_atoi(const char* s, int64_t* out) {
    const char* p = s;
    int neg = 0;
    if (*p == '+' || *p == '-') { neg = *p == '-'; p++; }
    if (!*p) return -1;
    int64_t v = 0;
    for (; *p; p++) {
        if (*p < '0' || *p > '9') return -1;
        if (v > (INT64_MAX - (*p - '0')) / 10) return -1;
        v = v * 10 + (*p - '0');
    }
    *out = neg ? -v : v;
    return 0;
}

/* strings.FieldsFunc(b, r == '\n'): iterate non-empty lines */
typedef struct { char* p; } line_iter;
static char* next_line(line_iter* it) {
    while (*it->p == '\n') it->p++;
    if (!*it->p) return NULL;
    char* st = it->p;
    while (*it->p && *it->p != '\n') it->p++;
    if (*it->p) *it->p++ = 0;
    return st;
}

/* test_common.go:29-68 readTopologyFile */
int orc_read_topology_text(orc_sim* s, char* text) {
    line_iter it = {text};
    char* line;
    int64_t left = -1;
    while ((line = next_line(&it))) {
        if (line[0] == '#') continue;
        if (left < 0) {
            if (go_atoi(line, &left)) return ORC_ERR_PARSE;
            continue;
        }
        char* f[3];
        if (go_fields(line, f, 3) != 2) return ORC_ERR_PARSE;
        if (left > 0) {
            int64_t tok;
            if (go_atoi(f[1], &tok)) return ORC_ERR_PARSE;
            if (orc_add_node(s, f[0], tok)) return ORC_ERR_API;
            left--;
        } else if (orc_add_link(s, f[0], f[1])) {
            return ORC_ERR_API;
        }
    }
    return ORC_OK;
}

int orc_read_topology(orc_sim* s, const char* path) {
    char* b = read_file(path, NULL);
    if (!b) return ORC_ERR_PARSE;
    int rc = orc_read_topology_text(s, b);
    free(b);
    return rc;
}

/* collect every completed, uncollected snapshot (the select at test_common.go:125-127) */
static int collect_ready(orc_sim* s) {
    int got = 0;
    for (int sid = 0; sid < s->next_snapshot_id; sid++)
        if (!s->collected[sid] && orc_snapshot_complete(s, sid)) { s->collected[sid] = 1; got++; }
    return got;
}

static int drain_events(orc_sim* s, int num_snapshots, int64_t max_drain_ticks);

/* test_common.go:79-140 readEventsFile, with the drain loop and maxDelay+1 ticks.
 * max_drain_ticks bounds the drain (the reference would tick forever): HANG. */
int orc_read_events_text(orc_sim* s, char* text, int64_t max_drain_ticks) {
    line_iter it = {text};
    char* line;
    int num_snapshots = 0;
    while ((line = next_line(&it))) {
        if (strcmp(line, "#") == 0) continue; /* strings.HasPrefix("#", line) (sic) */
        char* f[8];
        int nf = go_fields(line, f, 8);
        if (nf == 0) return ORC_ERR_PARSE; /* parts[0] index panic */
        int rc = ORC_OK;
        if (strcmp(f[0], "send") == 0) {
            int64_t n;
            if (nf < 4 || go_atoi(f[3], &n)) return ORC_ERR_PARSE;
            rc = orc_send_tokens(s, f[1], f[2], n);
        } else if (strcmp(f[0], "snapshot") == 0) {
            if (nf < 2) return ORC_ERR_PARSE;
            num_snapshots++;
            rc = orc_start_snapshot(s, f[1], NULL);
        } else if (strcmp(f[0], "tick") == 0) {
            int64_t n = 1;
            if (nf > 1 && go_atoi(f[1], &n)) return ORC_ERR_PARSE;
            for (int64_t i = 0; i < n && rc == ORC_OK; i++) rc = orc_tick(s);
        } else {
            return ORC_ERR_PARSE; /* log.Fatal("Unknown event command") */
        }
        if (rc < 0) return rc;
        if (rc > 0) return rc; /* per-instance fatal: the reference process exits */
    }
    return drain_events(s, num_snapshots, max_drain_ticks);
}

/* test_common.go:123-137: tick until every snapshot started by the file has been
 * collected, then maxDelay+1 more ticks */
static int drain_events(orc_sim* s, int num_snapshots, int64_t max_drain_ticks) {
    num_snapshots -= collect_ready(s);
    s->drain_ticks = 0;
    while (num_snapshots > 0) {
        if (s->drain_ticks >= max_drain_ticks) { s->status = ORC_HANG; return ORC_HANG; }
        int rc = orc_tick(s);
        s->drain_ticks++;
        if (rc) return rc;
        num_snapshots -= collect_ready(s);
    }
    for (int i = 0; i < MAX_DELAY + 1; i++) {
        int rc = orc_tick(s);
        if (rc) return rc;
    }
    return ORC_OK;
}

/* The drain of readEventsFile (test_common.go:123-137) on its own, after a program run
 * (orc_run_program): tick until every snapshot not yet collected has completed, then
 * maxDelay+1 more ticks. */
int orc_drain(orc_sim* s, int64_t max_drain_ticks) {
    if (s->status) return s->status;
    int pending = 0;
    for (int sid = 0; sid < s->next_snapshot_id; sid++) pending += !s->collected[sid];
    return drain_events(s, pending, max_drain_ticks);
}

int orc_read_events(orc_sim* s, const char* path, int64_t max_drain_ticks) {
    char* b = read_file(path, NULL);
    if (!b) return ORC_ERR_PARSE;
    int rc = orc_read_events_text(s, b, max_drain_ticks);
    free(b);
    return rc;
}

/* ------------------------------------------------------------------------- */
/* Batch runner: one independent simulation per instance, pthreads (cpu_baseline) */
/* ------------------------------------------------------------------------- */
typedef struct {
    const char* top;
    const char* events;
    const uint8_t* sched; /* [n][draws] or NULL -> Go seeds */
    int64_t draws;
    int64_t seed_base;
    int64_t lo, hi;
    int64_t max_drain;
    /* per instance outputs */
    int32_t* status;
    int64_t* ticks;
    int64_t* counters; /* [n][7] */
    uint64_t* hash;    /* [n] sum of completed snapshot hashes */
    int err;
} batch_job;

static void* batch_worker(void* arg) {
    batch_job* j = (batch_job*)arg;
    size_t tl = strlen(j->top), el = strlen(j->events);
    char* tb = (char*)xrealloc(NULL, tl + 1);
    char* eb = (char*)xrealloc(NULL, el + 1);
    for (int64_t i = j->lo; i < j->hi; i++) {
        orc_sim* s = orc_new();
        memcpy(tb, j->top, tl + 1);
        if (orc_read_topology_text(s, tb)) { j->err = 1; orc_free(s); break; }
        if (j->sched) orc_use_schedule(s, j->sched + i * j->draws, j->draws);
        else orc_seed_go(s, j->seed_base + i);
        memcpy(eb, j->events, el + 1);
        int rc = orc_read_events_text(s, eb, j->max_drain);
        if (rc < 0) { j->err = 1; orc_free(s); break; }
        if (j->status) j->status[i] = s->status;
        if (j->ticks) j->ticks[i] = s->time;
        if (j->counters) orc_counters_get(s, j->counters + 7 * i);
        if (j->hash) {
            uint64_t h = 0;
            for (int sid = 0; sid < s->next_snapshot_id; sid++) h += orc_snapshot_hash(s, sid);
            j->hash[i] = h;
        }
        orc_free(s);
    }
    free(tb); free(eb);
    return NULL;
}

/* Run instances [0, n) of (top, events); returns wall seconds or <0 on error. */
double orc_run_batch(const char* top_text, const char* events_text, int64_t n,
                     const uint8_t* sched, int64_t draws, int64_t seed_base,
                     int64_t max_drain, int threads, int32_t* status, int64_t* ticks,
                     int64_t* counters, uint64_t* hash) {
    if (threads < 1) threads = 1;
    batch_job* jobs = (batch_job*)calloc((size_t)threads, sizeof(batch_job));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < threads; t++) {
        batch_job* j = &jobs[t];
        j->top = top_text; j->events = events_text; j->sched = sched; j->draws = draws;
        j->seed_base = seed_base; j->max_drain = max_drain;
        j->lo = n * t / threads; j->hi = n * (t + 1) / threads;
        j->status = status; j->ticks = ticks; j->counters = counters; j->hash = hash;
        pthread_create(&th[t], NULL, batch_worker, j);
    }
    int err = 0;
    for (int t = 0; t < threads; t++) { pthread_join(th[t], NULL); err |= jobs[t].err; }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(jobs); free(th);
    if (err) return -1.0;
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ------------------------------------------------------------------------- */
/* Prepared batch runner (bench.py cpu_baseline): the topology and the event    */
/* file are parsed ONCE, outside the timed region -- as the GPU engine gets them */
/* resident before timing -- and each thread resets one simulator per instance  */
/* instead of re-parsing and re-allocating it.  The simulation itself is the    */
/* same literal restatement (orc_tick, send_tokens_idx, start_snapshot_idx).    */
/* ------------------------------------------------------------------------- */
enum { PEV_SEND = 1, PEV_SNAP = 2, PEV_TICK = 3 };
typedef struct { int kind, a, b; int64_t n; } prep_event; /* node indices (insertion order) */

/* Back to the state readTopologyFile left (sim.go:28-56): initial tokens, empty
 * queues, no snapshots, time 0.  Buffers are kept for reuse. */
static void orc_reset(orc_sim* s, const int64_t* init_tokens) {
    for (int i = 0; i < s->n_nodes; i++) {
        orc_node* n = &s->nodes[i];
        n->tokens = init_tokens[i];
        for (int k = 0; k < n->n_snaps; k++) {
            orc_local* l = &n->snaps[k];
            if (!l->exists) continue;
            free(l->is_link_recording);
            for (int j = 0; j < n->n_in; j++) free(l->incoming[j].v);
            free(l->incoming);
            l->exists = 0;
        }
        n->n_snaps = 0;
    }
    for (int i = 0; i < s->n_links; i++) { s->links[i].q.len = 0; s->links[i].q.head = 0; }
    for (int i = 0; i < s->cap_sids; i++) {
        s->completed_count[i] = 0; s->collected[i] = 0; s->completion_tick[i] = -1;
    }
    s->time = 0;
    s->next_snapshot_id = 0;
    s->status = 0;
    s->drain_ticks = 0;
    s->n_log = 0;
    s->sched_pos = 0;
    memset(&s->cnt, 0, sizeof(s->cnt));
}

/* The event loop of readEventsFile (test_common.go:92-121) over prepared events, then
 * its drain (test_common.go:123-137). */
static int run_prepared(orc_sim* s, const prep_event* ev, int64_t n_ev, int64_t max_drain) {
    int num_snapshots = 0;
    for (int64_t i = 0; i < n_ev; i++) {
        const prep_event* e = &ev[i];
        int rc = ORC_OK;
        if (e->kind == PEV_SEND) {
            rc = s->status ? s->status : send_tokens_idx(s, e->a, e->b, e->n);
        } else if (e->kind == PEV_SNAP) {
            num_snapshots++;
            rc = s->status ? s->status : start_snapshot_idx(s, e->a, NULL);
        } else {
            for (int64_t k = 0; k < e->n && rc == ORC_OK; k++) rc = orc_tick(s);
        }
        if (rc) return rc;
    }
    return drain_events(s, num_snapshots, max_drain);
}

typedef struct {
    const char* top;
    const prep_event* ev;
    int64_t n_ev;
    int64_t seed_base, lo, hi, max_drain;
    int32_t* status;
    int64_t* ticks;
    int64_t* counters;
    uint64_t* hash;
    pthread_barrier_t* bar;
    struct timespec t0, t1;
    int err;
} prep_job;

static void* prep_worker(void* arg) {
    prep_job* j = (prep_job*)arg;
    /* untimed: this thread's simulator from the topology text */
    char* tb = strdup(j->top);
    orc_sim* s = orc_new();
    if (orc_read_topology_text(s, tb)) j->err = 1;
    free(tb);
    int64_t* init = (int64_t*)xrealloc(NULL, sizeof(int64_t) * (size_t)(s->n_nodes ? s->n_nodes : 1));
    for (int i = 0; i < s->n_nodes; i++) init[i] = s->nodes[i].tokens;
    pthread_barrier_wait(j->bar);
    clock_gettime(CLOCK_MONOTONIC, &j->t0);
    for (int64_t i = j->lo; i < j->hi && !j->err; i++) {
        orc_reset(s, init);
        orc_seed_go(s, j->seed_base + i); /* rand.Seed(seed_base + i), snapshot_test.go:20 */
        if (run_prepared(s, j->ev, j->n_ev, j->max_drain) < 0) { j->err = 1; break; }
        if (j->status) j->status[i] = s->status;
        if (j->ticks) j->ticks[i] = s->time;
        if (j->counters) orc_counters_get(s, j->counters + 7 * i);
        if (j->hash) {
            uint64_t h = 0;
            for (int sid = 0; sid < s->next_snapshot_id; sid++) h += orc_snapshot_hash(s, sid);
            j->hash[i] = h;
        }
    }
    clock_gettime(CLOCK_MONOTONIC, &j->t1);
    free(init);
    orc_free(s);
    return NULL;
}

static double ts_sec(struct timespec t) { return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec; }

/* Instances [0, n) of (top, events) with Go seeds seed_base + i, on `threads` threads.
 * Returns the wall seconds of the simulations alone (from the release of the start
 * barrier to the last thread's end), or < 0 on a parse/API error.  hash may be NULL
 * (not timed work of the engine either). */
double orc_run_batch_prepared(const char* top_text, const char* events_text, int64_t n, int64_t seed_base,
                              int64_t max_drain, int threads, int32_t* status, int64_t* ticks,
                              int64_t* counters, uint64_t* hash) {
    if (threads < 1) threads = 1;
    /* parse the events once against a scratch simulator (node indices = insertion order) */
    orc_sim* s = orc_new();
    char* tb = strdup(top_text);
    int bad = orc_read_topology_text(s, tb) != ORC_OK;
    free(tb);
    char* eb = strdup(events_text);
    line_iter it = {eb};
    char* line;
    prep_event* ev = NULL;
    int64_t n_ev = 0, cap_ev = 0;
    while (!bad && (line = next_line(&it))) {
        if (strcmp(line, "#") == 0) continue; /* test_common.go:90 (sic) */
        char* f[8];
        int nf = go_fields(line, f, 8);
        prep_event e = {0, -1, -1, 0};
        if (nf == 0) { bad = 1; break; }
        if (strcmp(f[0], "send") == 0) {
            if (nf < 4 || go_atoi(f[3], &e.n)) { bad = 1; break; }
            e.kind = PEV_SEND; e.a = find_node(s, f[1]); e.b = find_node(s, f[2]);
            if (e.a < 0) { bad = 1; break; }
        } else if (strcmp(f[0], "snapshot") == 0) {
            if (nf < 2) { bad = 1; break; }
            e.kind = PEV_SNAP; e.a = find_node(s, f[1]);
            if (e.a < 0) { bad = 1; break; }
        } else if (strcmp(f[0], "tick") == 0) {
            e.kind = PEV_TICK; e.n = 1;
            if (nf > 1 && go_atoi(f[1], &e.n)) { bad = 1; break; }
        } else {
            bad = 1; break;
        }
        if (n_ev == cap_ev) {
            cap_ev = cap_ev ? 2 * cap_ev : 64;
            ev = (prep_event*)xrealloc(ev, sizeof(prep_event) * (size_t)cap_ev);
        }
        ev[n_ev++] = e;
    }
    free(eb);
    orc_free(s);
    if (bad) { free(ev); return -1.0; }
    prep_job* jobs = (prep_job*)calloc((size_t)threads, sizeof(prep_job));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)threads);
    for (int t = 0; t < threads; t++) {
        prep_job* j = &jobs[t];
        j->top = top_text; j->ev = ev; j->n_ev = n_ev; j->seed_base = seed_base; j->max_drain = max_drain;
        j->lo = n * t / threads; j->hi = n * (t + 1) / threads;
        j->status = status; j->ticks = ticks; j->counters = counters; j->hash = hash; j->bar = &bar;
        pthread_create(&th[t], NULL, prep_worker, j);
    }
    int err = 0;
    double t0 = 1e300, t1 = 0;
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        err |= jobs[t].err;
        if (ts_sec(jobs[t].t0) < t0) t0 = ts_sec(jobs[t].t0);
        if (ts_sec(jobs[t].t1) > t1) t1 = ts_sec(jobs[t].t1);
    }
    pthread_barrier_destroy(&bar);
    free(jobs); free(th); free(ev);
    return err ? -1.0 : t1 - t0;
}

/* ------------------------------------------------------------------------- */
/* Synthetic large-graph driver         */
/* ------------------------------------------------------------------------- */
/* Build a topology from ranks: node r gets id "N" + r zero-padded to `width`
 * digits (lexicographic order == numeric order, so rank r is sorted position r),
 * then AddLink(src[i], dst[i]) in edge order -- the same calls readTopologyFile
 * would make (test_common.go:29-68), without re-sorting after every AddNode. */
int orc_build_graph(orc_sim* s, int n, const int64_t* tokens, int64_t m, const int32_t* src,
                    const int32_t* dst, int width) {
    if (s->n_nodes) return ORC_ERR_API;
    s->nodes = (orc_node*)xrealloc(s->nodes, sizeof(orc_node) * (size_t)(n ? n : 1));
    s->cap_nodes = n ? n : 1;
    char buf[32];
    for (int r = 0; r < n; r++) {
        orc_node* nd = &s->nodes[r];
        memset(nd, 0, sizeof(*nd));
        snprintf(buf, sizeof buf, "N%0*d", width, r);
        nd->id = strdup(buf);
        nd->tokens = tokens[r];
    }
    s->n_nodes = n;
    resort(s);
    for (int r = 0; r < n; r++)
        if (s->sorted[r] != r) return ORC_ERR_API; /* width too small for lexicographic == numeric */
    for (int64_t i = 0; i < m; i++) {
        int a = src[i], b = dst[i];
        if (a < 0 || b < 0 || a >= n || b >= n) return ORC_ERR_API;
        if (a == b) continue; /* node.go:88-90 */
        orc_node* na = &s->nodes[a];
        int dup = 0;
        for (int k = 0; k < na->n_out && !dup; k++) dup = s->links[na->out_links[k]].dest == b;
        if (dup) continue; /* map assignment: a fresh queue, nothing pushed yet */
        if (s->n_links == s->cap_links) {
            s->cap_links = s->cap_links ? 2 * s->cap_links : 16;
            s->links = (orc_link*)xrealloc(s->links, sizeof(orc_link) * (size_t)s->cap_links);
        }
        int li = s->n_links++;
        memset(&s->links[li], 0, sizeof(orc_link));
        s->links[li].src = a;
        s->links[li].dest = b;
        insert_sorted(s, &na->out_links, &na->n_out, &na->cap_out, li, 1);
        orc_node* nb = &s->nodes[b];
        insert_sorted(s, &nb->in_links, &nb->n_in, &nb->cap_in, li, 0);
    }
    return ORC_OK;
}

/* The synthetic traffic of one step: every node, in sorted order, that holds tokens
 * and has out-links sends ONE token to out-link j with probability thresh / 2^32,
 * both decided by the counter hash of (seed, step, rank).  Each send is the
 * reference's SendTokens (node.go:112-131) with n = 1, so it draws one delay. */
int orc_traffic_sends(orc_sim* s, uint64_t seed, uint32_t thresh, int64_t step) {
    if (s->status) return s->status;
    for (int a = 0; a < s->n_nodes; a++) {
        int v = s->sorted[a];
        orc_node* n = &s->nodes[v];
        if (n->tokens <= 0 || n->n_out == 0) continue;
        uint64_t x = orc_counter_hash(seed, (uint64_t)step, (uint64_t)a);
        if ((uint32_t)x >= thresh) continue;
        int j = (int)(((x >> 32) * (uint64_t)n->n_out) >> 32);
        int rc = send_tokens_idx(s, v, s->links[n->out_links[j]].dest, 1);
        if (rc) return rc;
    }
    return ORC_OK;
}

/* A synthetic program: for step k in [0, steps): traffic sends (k < traffic_steps),
 * then the snapshots scheduled at step k in list order (StartSnapshot on rank
 * snap_rank[i], sim.go:105-123), then Tick (sim.go:71-95).  Nodes are ranks. */
int orc_run_program(orc_sim* s, int64_t steps, uint64_t traffic_seed, uint32_t thresh,
                    int64_t traffic_steps, int n_snap, const int32_t* snap_step,
                    const int32_t* snap_rank) {
    int si = 0;
    for (int64_t k = 0; k < steps; k++) {
        int rc = ORC_OK;
        if (k < traffic_steps) rc = orc_traffic_sends(s, traffic_seed, thresh, k);
        while (rc == ORC_OK && si < n_snap && snap_step[si] == k) {
            rc = start_snapshot_idx(s, s->sorted[snap_rank[si]], NULL);
            si++;
        }
        while (si < n_snap && snap_step[si] < k) si++;
        if (rc == ORC_OK) rc = orc_tick(s);
        if (rc) return rc;
    }
    return ORC_OK;
}

/* Snapshot sid by channel: tokens[N] in rank order; channels in (src rank, dest rank)
 * order; the recorded messages of channel c are vals[off[c] .. off[c+1]) in recording
 * order.  Works for incomplete snapshots too (what has been recorded so far; nodes
 * without the local snapshot get tokens -1 and empty channels).  Returns total count
 * (vals written only below cap). */
int64_t orc_collect_channels(const orc_sim* s, int sid, int64_t* tokens, int64_t* off, int64_t* vals,
                             int64_t cap) {
    int64_t m = 0, c = 0;
    for (int a = 0; a < s->n_nodes; a++) {
        const orc_node* n = &s->nodes[s->sorted[a]];
        const orc_local* l = local_snap((orc_node*)n, sid);
        tokens[a] = l ? l->num_tokens_in_node : -1;
    }
    for (int a = 0; a < s->n_nodes; a++) {
        const orc_node* src = &s->nodes[s->sorted[a]];
        for (int k = 0; k < src->n_out; k++, c++) {
            const orc_link* lk = &s->links[src->out_links[k]];
            const orc_local* l = local_snap(&s->nodes[lk->dest], sid);
            off[c] = m;
            if (!l) continue;
            const i64vec* v = &l->incoming[in_index(s, lk->dest, lk->src)];
            for (int64_t q = 0; q < v->n; q++, m++)
                if (m < cap) vals[m] = v->v[q];
        }
    }
    off[c] = m;
    return m;
}

int orc_num_links(const orc_sim* s) { return s->n_links; }

/* Out-channel queue depths in channel order (diagnostics: FIFO sizing). */
void orc_queue_depths(const orc_sim* s, int64_t* out) {
    int64_t c = 0;
    for (int a = 0; a < s->n_nodes; a++) {
        const orc_node* src = &s->nodes[s->sorted[a]];
        for (int k = 0; k < src->n_out; k++, c++) out[c] = s->links[src->out_links[k]].q.len;
    }
}
