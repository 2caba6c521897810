/*
 * sentinel_oracle.c -- CPU restatement of Sentinel's sliding-window token-decision path.
 *
 * TEST INFRASTRUCTURE ONLY (parity checker + "port" CPU baseline).  See sentinel_oracle.h.
 * Compiled with -O2 -ffp-contract=off and no fast-math so every double operation is one IEEE
 * operation in Java source order (JLS 15.17-15.18; strictfp is the default since Java 17 and
 * HotSpot on x86-64 SSE2 already behaves that way for Java 7/8).
 *
 * Reference paths (under /root/reference):
 *   LA  = sentinel-core/src/main/java/com/alibaba/csp/sentinel/slots/statistic/base/LeapArray.java
 *   CM  = sentinel-cluster/sentinel-cluster-server-default/src/main/java/com/alibaba/csp/sentinel/
 *         cluster/flow/statistic/metric/ClusterMetric.java
 *   CMLA= .../cluster/flow/statistic/metric/ClusterMetricLeapArray.java
 *   CFC = .../cluster/flow/ClusterFlowChecker.java
 *   DTS = .../cluster/flow/DefaultTokenService.java
 *   RL  = .../cluster/flow/statistic/limit/RequestLimiter.java
 *   GRL = .../cluster/flow/statistic/limit/GlobalRequestLimiter.java
 *   CPM = .../cluster/flow/statistic/metric/ClusterParamMetric.java
 *   CPFC= .../cluster/flow/ClusterParamFlowChecker.java
 *   SCFC= sentinel-cluster/sentinel-cluster-server-envoy-rls/.../rls/flow/SimpleClusterFlowChecker.java
 *   SN  = sentinel-core/.../node/StatisticNode.java
 *   DC  = sentinel-core/.../slots/block/flow/controller/DefaultController.java
 *   PFC = sentinel-extension/sentinel-parameter-flow-control/.../slots/block/flow/param/ParamFlowChecker.java
 */
#include "sentinel_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ Java numerics */

/* JLS 5.1.3 narrowing double -> int: NaN -> 0, saturate at the int range, else truncate. */
int32_t orc_java_d2i(double d) {
    if (d != d) return 0;
    if (d >= 2147483647.0) return INT32_MAX;
    if (d <= -2147483648.0) return INT32_MIN;
    return (int32_t)d;
}

int64_t orc_java_d2l(double d) {
    if (d != d) return 0;
    if (d >= 9223372036854775807.0) return INT64_MAX;
    if (d <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)d;
}

/* java.lang.String.hashCode: s[0]*31^(n-1) + ... with int overflow. */
int32_t orc_java_string_hash(const uint16_t *s, int64_t n) {
    uint32_t h = 0;
    for (int64_t i = 0; i < n; i++) h = 31u * h + (uint32_t)s[i];
    return (int32_t)h;
}

static int64_t wrap_add64(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
static int64_t wrap_mul64(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }

/* ------------------------------------------------------------------ LeapArray core */
/* The slot array of LA:41-78: sampleCount WindowWraps {windowStart, value}. */
typedef struct {
    int n, win, interval;
    double interval_sec;     /* LA:74 intervalInMs / 1000.0 */
    int64_t *start;
    uint8_t *present;
} leap;

enum { LA_SAME = 0, LA_NEW = 1, LA_RESET = 2, LA_DETACHED = 3, LA_NULL = 4 };

static void leap_init(leap *a, int n, int interval_ms) {
    a->n = n;
    a->interval = interval_ms;
    a->win = interval_ms / n;                 /* LA:72 */
    a->interval_sec = interval_ms / 1000.0;   /* LA:74 */
    a->start = (int64_t *)calloc((size_t)n, sizeof(int64_t));
    a->present = (uint8_t *)calloc((size_t)n, 1);
}

static void leap_free(leap *a) { free(a->start); free(a->present); }

/* LA:112-124 calculateTimeIdx */
static int leap_idx(const leap *a, int64_t t) { return (int)((t / a->win) % a->n); }

/* LA:149-248 currentWindow(t), single-threaded: the CAS always wins and tryLock always succeeds.
 * Returns the action; *idx = slot.  The caller applies newEmptyBucket / resetWindowTo. */
static int leap_locate(leap *a, int64_t t, int *idx) {
    if (t < 0) return LA_NULL;                        /* LA:150-152 */
    int i = leap_idx(a, t);
    int64_t ws = t - t % a->win;                      /* LA:140 */
    *idx = i;
    if (!a->present[i]) {                             /* LA:172-194 */
        a->present[i] = 1;
        a->start[i] = ws;
        return LA_NEW;
    }
    if (ws == a->start[i]) return LA_SAME;            /* LA:195-209 */
    if (ws > a->start[i]) {                           /* LA:210-240 resetWindowTo */
        a->start[i] = ws;                             /* WindowWrap.resetTo */
        return LA_RESET;
    }
    return LA_DETACHED;                               /* LA:241-246: a fresh, unshared wrap */
}

/* LA:316-318 isWindowDeprecated(time, w) */
static int leap_deprecated(const leap *a, int64_t t, int i) { return t - a->start[i] > a->interval; }

/* ------------------------------------------------------------------ ClusterMetric */
struct orc_cluster_metric {
    leap la;
    int64_t *c;                 /* n x 7 ClusterMetricBucket counters */
    int64_t occ[ORC_NEVENTS];   /* CMLA:129 occupyCounter */
    int has_occupied;           /* CMLA:130 */
    int64_t scratch[ORC_NEVENTS];
};

orc_cluster_metric *orc_cm_new(int sample_count, int interval_ms) {
    if (sample_count <= 0 || interval_ms <= 0 || interval_ms % sample_count != 0) return NULL; /* CM:33-35 */
    orc_cluster_metric *m = (orc_cluster_metric *)calloc(1, sizeof(*m));
    leap_init(&m->la, sample_count, interval_ms);
    m->c = (int64_t *)calloc((size_t)sample_count * ORC_NEVENTS, sizeof(int64_t));
    return m;
}

void orc_cm_free(orc_cluster_metric *m) {
    if (!m) return;
    leap_free(&m->la);
    free(m->c);
    free(m);
}

/* LA currentWindow + CMLA:141-161 (newEmptyBucket / resetWindowTo + transferOccupyToBucket). */
static int64_t *cm_current(orc_cluster_metric *m, int64_t t) {
    int i = 0;
    int act = leap_locate(&m->la, t, &i);
    if (act == LA_NULL) return NULL;
    if (act == LA_DETACHED) {
        memset(m->scratch, 0, sizeof(m->scratch));
        return m->scratch;
    }
    int64_t *b = m->c + (size_t)i * ORC_NEVENTS;
    if (act == LA_NEW) {
        memset(b, 0, sizeof(int64_t) * ORC_NEVENTS);  /* CMLA:142-144 new ClusterMetricBucket() */
    } else if (act == LA_RESET) {
        memset(b, 0, sizeof(int64_t) * ORC_NEVENTS);  /* CMLA:149 reset() */
        if (m->has_occupied) {                        /* CMLA:154-161 */
            b[ORC_OCCUPIED_PASS] = wrap_add64(b[ORC_OCCUPIED_PASS], m->occ[ORC_PASS]);
            b[ORC_PASS] = wrap_add64(b[ORC_PASS], m->occ[ORC_PASS]);
            m->occ[ORC_PASS] = 0;
            b[ORC_PASS_REQUEST] = wrap_add64(b[ORC_PASS_REQUEST], m->occ[ORC_PASS_REQUEST]);
            m->occ[ORC_PASS_REQUEST] = 0;
            m->has_occupied = 0;
        }
    }
    return b;
}

/* CM:39-41 */
void orc_cm_add(orc_cluster_metric *m, int64_t t, int event, int64_t count) {
    int64_t *b = cm_current(m, t);
    if (b) b[event] = wrap_add64(b[event], count);
}

/* CM:43-45 */
int64_t orc_cm_get_current_count(orc_cluster_metric *m, int64_t t, int event) {
    int64_t *b = cm_current(m, t);
    return b ? b[event] : 0;
}

/* CM:53-62: currentWindow(); sum over values() (LA:375-390). */
int64_t orc_cm_get_sum(orc_cluster_metric *m, int64_t t, int event) {
    cm_current(m, t);
    if (t < 0) return 0;
    int64_t sum = 0;
    for (int i = 0; i < m->la.n; i++) {
        if (!m->la.present[i] || leap_deprecated(&m->la, t, i)) continue;
        sum = wrap_add64(sum, m->c[(size_t)i * ORC_NEVENTS + event]);
    }
    return sum;
}

/* CM:70-72: long / double */
double orc_cm_get_avg(orc_cluster_metric *m, int64_t t, int event) {
    return (double)orc_cm_get_sum(m, t, event) / m->la.interval_sec;
}

/* CMLA:181-190 getFirstCountOfWindow via LA:399-409 getValidHead(t). */
static int64_t cm_first_count(orc_cluster_metric *m, int64_t t, int event) {
    int i = leap_idx(&m->la, t + m->la.win);
    if (!m->la.present[i] || leap_deprecated(&m->la, t, i)) return 0;
    return m->c[(size_t)i * ORC_NEVENTS + event];
}

/* CM:79-98 */
int orc_cm_try_occupy_next(orc_cluster_metric *m, int64_t t, int event, int acquire, double threshold) {
    double latest = orc_cm_get_avg(m, t, ORC_PASS);
    int64_t head = cm_first_count(m, t, event);
    int64_t occupied = m->occ[event];
    /* latestQps + (acquireCount + occupiedCount) - headPass <= threshold  (int+long -> long) */
    int64_t inner = wrap_add64((int64_t)acquire, occupied);
    double lhs = (latest + (double)inner) - (double)head;
    if (!(lhs <= threshold)) return 0;
    m->occ[ORC_PASS] = wrap_add64(m->occ[ORC_PASS], acquire);        /* CMLA:171-175 */
    m->occ[ORC_PASS_REQUEST] = wrap_add64(m->occ[ORC_PASS_REQUEST], 1);
    m->has_occupied = 1;
    orc_cm_add(m, t, ORC_WAITING, acquire);
    return 1000 / m->la.n;                                            /* CM:86 */
}

void orc_cm_dump(const orc_cluster_metric *m, int64_t *out) {
    int n = m->la.n;
    for (int i = 0; i < n; i++) {
        int64_t *o = out + (size_t)i * (1 + ORC_NEVENTS);
        o[0] = m->la.present[i] ? m->la.start[i] : -1;
        for (int e = 0; e < ORC_NEVENTS; e++) o[1 + e] = m->la.present[i] ? m->c[(size_t)i * ORC_NEVENTS + e] : 0;
    }
    int64_t *o = out + (size_t)n * (1 + ORC_NEVENTS);
    for (int e = 0; e < ORC_NEVENTS; e++) o[e] = m->occ[e];
    o[ORC_NEVENTS] = m->has_occupied;
}

int orc_cm_list_count(const orc_cluster_metric *m, int64_t t) {
    int k = 0;
    for (int i = 0; i < m->la.n; i++)
        if (m->la.present[i] && !leap_deprecated(&m->la, t, i)) k++;
    return k;
}

int64_t orc_cm_first_count(orc_cluster_metric *m, int64_t t, int event) { return cm_first_count(m, t, event); }

int64_t orc_cm_window_start(orc_cluster_metric *m, int64_t t) {
    int i = 0;
    if (t < 0) return -1;
    int64_t *b = cm_current(m, t);
    (void)b;
    i = leap_idx(&m->la, t);
    return m->la.start[i] == t - t % m->la.win ? m->la.start[i] : t - t % m->la.win;
}

/* ------------------------------------------------------------------ RequestLimiter */
/* RL:35-37: UnaryLeapArray(10, 1000) (core/.../base/UnaryLeapArray.java:21-38). */
struct orc_limiter {
    leap la;
    int64_t *v;
    double qps_allowed;
};

orc_limiter *orc_limiter_new(double qps_allowed) {
    orc_limiter *l = (orc_limiter *)calloc(1, sizeof(*l));
    leap_init(&l->la, 10, 1000);
    l->v = (int64_t *)calloc(10, sizeof(int64_t));
    l->qps_allowed = qps_allowed;
    return l;
}

void orc_limiter_free(orc_limiter *l) {
    if (!l) return;
    leap_free(&l->la);
    free(l->v);
    free(l);
}

static int64_t lim_scratch;
static int64_t *lim_current(orc_limiter *l, int64_t t) {
    int i = 0;
    int act = leap_locate(&l->la, t, &i);
    if (act == LA_NULL) return NULL;
    if (act == LA_DETACHED) { lim_scratch = 0; return &lim_scratch; }
    if (act == LA_NEW || act == LA_RESET) l->v[i] = 0;   /* UnaryLeapArray.java:28-37 */
    return &l->v[i];
}

void orc_limiter_add(orc_limiter *l, int64_t t, int x) {   /* RL:49-51 */
    int64_t *p = lim_current(l, t);
    if (p) *p = wrap_add64(*p, x);
}

int64_t orc_limiter_get_sum(orc_limiter *l, int64_t t) {   /* RL:53-62 */
    lim_current(l, t);
    int64_t s = 0;
    for (int i = 0; i < l->la.n; i++)
        if (l->la.present[i] && !leap_deprecated(&l->la, t, i)) s = wrap_add64(s, l->v[i]);
    return s;
}

double orc_limiter_get_qps(orc_limiter *l, int64_t t) {    /* RL:64-66 */
    return (double)orc_limiter_get_sum(l, t) / l->la.interval_sec;
}

int orc_limiter_can_pass(orc_limiter *l, int64_t t) {      /* RL:72-74 */
    return orc_limiter_get_qps(l, t) + 1 <= l->qps_allowed;
}

int orc_limiter_try_pass(orc_limiter *l, int64_t t) {      /* RL:81-87 */
    if (orc_limiter_can_pass(l, t)) {
        orc_limiter_add(l, t, 1);
        return 1;
    }
    return 0;
}

/* ------------------------------------------------------------------ exact key->count map */
typedef struct {
    uint64_t *k;
    int64_t *v;
    uint8_t *used;
    int64_t cap, size;
} kvmap;

static void kv_init(kvmap *m) { memset(m, 0, sizeof(*m)); }
static void kv_free(kvmap *m) { free(m->k); free(m->v); free(m->used); memset(m, 0, sizeof(*m)); }
static void kv_clear(kvmap *m) { if (m->used) memset(m->used, 0, (size_t)m->cap); m->size = 0; }

static uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
    return x;
}

static int64_t *kv_find(kvmap *m, uint64_t key) {
    if (!m->cap) return NULL;
    uint64_t h = mix64(key) & (uint64_t)(m->cap - 1);
    while (m->used[h]) {
        if (m->k[h] == key) return &m->v[h];
        h = (h + 1) & (uint64_t)(m->cap - 1);
    }
    return NULL;
}

static int64_t *kv_insert(kvmap *m, uint64_t key, int64_t init) {
    int64_t *p = kv_find(m, key);
    if (p) return p;
    if ((m->size + 1) * 2 > m->cap) {
        kvmap n;
        n.cap = m->cap ? m->cap * 2 : 16;
        n.size = 0;
        n.k = (uint64_t *)calloc((size_t)n.cap, sizeof(uint64_t));
        n.v = (int64_t *)calloc((size_t)n.cap, sizeof(int64_t));
        n.used = (uint8_t *)calloc((size_t)n.cap, 1);
        for (int64_t i = 0; i < m->cap; i++)
            if (m->used[i]) *kv_insert(&n, m->k[i], m->v[i]) = m->v[i];
        kv_free(m);
        *m = n;
    }
    uint64_t h = mix64(key) & (uint64_t)(m->cap - 1);
    while (m->used[h]) h = (h + 1) & (uint64_t)(m->cap - 1);
    m->used[h] = 1;
    m->k[h] = key;
    m->v[h] = init;
    m->size++;
    return &m->v[h];
}

/* ------------------------------------------------------------------ ClusterParamMetric */
/* Each bucket is a CacheMap<Object, LongAdder> (ClusterParameterLeapArray.java:40-49).  The LRU
 * eviction of ConcurrentLinkedHashMap (capacity 4000) is NOT restated: exact counters only, and
 * `overflow` records that a bucket exceeded its capacity (parity unpinned past that point). */
struct orc_param_metric {
    leap la;
    kvmap *b;
    kvmap scratch;
    int max_capacity;
    int overflow;
};

orc_param_metric *orc_pm_new(int sample_count, int interval_ms, int max_capacity) {
    if (sample_count <= 0 || interval_ms <= 0 || interval_ms % sample_count != 0 || max_capacity <= 0) return NULL;
    orc_param_metric *m = (orc_param_metric *)calloc(1, sizeof(*m));
    leap_init(&m->la, sample_count, interval_ms);
    m->b = (kvmap *)calloc((size_t)sample_count, sizeof(kvmap));
    kv_init(&m->scratch);
    m->max_capacity = max_capacity;
    return m;
}

void orc_pm_free(orc_param_metric *m) {
    if (!m) return;
    for (int i = 0; i < m->la.n; i++) kv_free(&m->b[i]);
    kv_free(&m->scratch);
    free(m->b);
    leap_free(&m->la);
    free(m);
}

static kvmap *pm_current(orc_param_metric *m, int64_t t) {
    int i = 0;
    int act = leap_locate(&m->la, t, &i);
    if (act == LA_NULL) return NULL;
    if (act == LA_DETACHED) { kv_clear(&m->scratch); return &m->scratch; }
    if (act == LA_NEW || act == LA_RESET) kv_clear(&m->b[i]);   /* new map / clear() */
    return &m->b[i];
}

void orc_pm_add_value(orc_param_metric *m, int64_t t, uint64_t key, int count) {   /* CPM:66-78 */
    kvmap *b = pm_current(m, t);
    if (!b) return;
    int64_t *p = kv_insert(b, key, 0);
    *p = wrap_add64(*p, count);
    if (b->size > m->max_capacity) m->overflow = 1;
}

int64_t orc_pm_get_sum(orc_param_metric *m, int64_t t, uint64_t key) {             /* CPM:46-60 */
    pm_current(m, t);
    int64_t s = 0;
    for (int i = 0; i < m->la.n; i++) {
        if (!m->la.present[i] || leap_deprecated(&m->la, t, i)) continue;
        int64_t *p = kv_find(&m->b[i], key);
        if (p) s = wrap_add64(s, *p);
    }
    return s;
}

double orc_pm_get_avg(orc_param_metric *m, int64_t t, uint64_t key) {              /* CPM:80-82 */
    return (double)orc_pm_get_sum(m, t, key) / m->la.interval_sec;
}

typedef struct { uint64_t k; int64_t v; int64_t ord; } kvent;
static int cmp_top(const void *pa, const void *pb) {
    const kvent *a = (const kvent *)pa, *b = (const kvent *)pb;
    /* CPM:107-113: (int) b - (int) a, descending by (int)value; ties keep insertion order. */
    int32_t ia = (int32_t)a->v, ib = (int32_t)b->v;
    int32_t d = (int32_t)((uint32_t)ib - (uint32_t)ia);
    if (d != 0) return d < 0 ? -1 : 1;
    return a->ord < b->ord ? -1 : (a->ord > b->ord);
}

int orc_pm_top_values(orc_param_metric *m, int64_t t, int number, uint64_t *keys, double *avgs) {  /* CPM:84-127 */
    if (number <= 0) return -1;
    pm_current(m, t);
    kvmap merged;
    kv_init(&merged);
    for (int i = 0; i < m->la.n; i++) {
        if (!m->la.present[i] || leap_deprecated(&m->la, t, i)) continue;
        for (int64_t j = 0; j < m->b[i].cap; j++) {
            if (!m->b[i].used[j]) continue;
            int64_t *p = kv_insert(&merged, m->b[i].k[j], 0);
            *p = wrap_add64(*p, m->b[i].v[j]);
        }
    }
    kvent *ents = (kvent *)calloc((size_t)(merged.size ? merged.size : 1), sizeof(kvent));
    int64_t ne = 0;
    for (int64_t j = 0; j < merged.cap; j++)
        if (merged.used[j]) { ents[ne].k = merged.k[j]; ents[ne].v = merged.v[j]; ents[ne].ord = ne; ne++; }
    /* Java HashMap iteration order is unspecified; sort ties by key for determinism. */
    for (int64_t a = 0; a < ne; a++) ents[a].ord = (int64_t)ents[a].k;
    qsort(ents, (size_t)ne, sizeof(kvent), cmp_top);
    int size = ne > number ? number : (int)ne;
    int out = 0;
    for (int i = 0; i < size; i++) {
        if (ents[i].v == 0) break;
        keys[out] = ents[i].k;
        avgs[out] = (double)ents[i].v / m->la.interval_sec;
        out++;
    }
    free(ents);
    kv_free(&merged);
    return out;
}

int orc_pm_overflowed(const orc_param_metric *m) { return m->overflow; }

/* ------------------------------------------------------------------ engine (DefaultTokenService) */
typedef struct {
    orc_param_rule r;
    orc_param_metric *pm;
} param_entry;

/* TokenCacheNodeManager's cache: tokenId -> record {flowId, acquireCount, alive} (one per engine; a
 * flow-sharded replay gives every thread its own). */
typedef struct {
    kvmap index;
    int64_t *fid;
    int32_t *acq;
    uint8_t *alive;
    int64_t n, cap, live;
} orc_tok;
static void tok_free(orc_tok *t);

struct orc_engine {
    orc_server_config cfg;
    orc_namespace *ns;
    orc_limiter **lim;
    int n_ns;
    orc_flow_rule *rules;       /* dense table: valid rules, one per flowId (first position, last content) */
    orc_cluster_metric **cm;    /* cm[i] = METRIC_MAP.get(rules[i].flowId) (owned by metric_map) */
    int n_rules;
    kvmap metric_map;           /* ClusterMetricStatistics.METRIC_MAP: flowId -> orc_cluster_metric* */
    param_entry *prules;        /* dense table of valid param rules; pm owned by param_metric_map */
    int n_prules;
    kvmap param_metric_map;     /* ClusterParamMetricStatistics.METRIC_MAP: flowId -> orc_param_metric* */
    uint64_t *hot_keys;
    int32_t *hot_counts;
    int n_hot;
    /* concurrency tokens (ConcurrentClusterFlowChecker) */
    kvmap now_calls;          /* flowId -> nowCalls (CurrentConcurrencyManager) */
    kvmap rule_by_fid;        /* flowId -> rule index (ClusterFlowRuleManager.getFlowRuleById) */
    orc_tok tok;              /* TokenCacheNodeManager */
};

orc_engine *orc_engine_new(const orc_server_config *cfg, const orc_namespace *ns, int n_ns) {
    orc_engine *e = (orc_engine *)calloc(1, sizeof(*e));
    e->cfg = *cfg;
    e->n_ns = n_ns;
    e->ns = (orc_namespace *)calloc((size_t)(n_ns > 0 ? n_ns : 1), sizeof(orc_namespace));
    e->lim = (orc_limiter **)calloc((size_t)(n_ns > 0 ? n_ns : 1), sizeof(orc_limiter *));
    for (int i = 0; i < n_ns; i++) {
        e->ns[i] = ns[i];
        /* GRL:32-37 initIfAbsent -> new RequestLimiter(maxAllowedQps) */
        if (ns[i].has_limiter) e->lim[i] = orc_limiter_new(ns[i].max_allowed_qps);
    }
    return e;
}

void orc_engine_free(orc_engine *e) {
    if (!e) return;
    for (int i = 0; i < e->n_ns; i++) orc_limiter_free(e->lim[i]);
    for (int64_t j = 0; j < e->metric_map.cap; j++)
        if (e->metric_map.used[j]) orc_cm_free((orc_cluster_metric *)(intptr_t)e->metric_map.v[j]);
    for (int64_t j = 0; j < e->param_metric_map.cap; j++)
        if (e->param_metric_map.used[j]) orc_pm_free((orc_param_metric *)(intptr_t)e->param_metric_map.v[j]);
    kv_free(&e->metric_map); kv_free(&e->param_metric_map);
    free(e->ns); free(e->lim); free(e->rules); free(e->cm); free(e->prules);
    free(e->hot_keys); free(e->hot_counts);
    kv_free(&e->now_calls); kv_free(&e->rule_by_fid);
    tok_free(&e->tok);
    free(e);
}

/* Remove `key` from a kvmap (backward-shift deletion keeps linear-probe chains intact). */
static void kv_erase(kvmap *m, uint64_t key) {
    if (!m->cap) return;
    const uint64_t mask = (uint64_t)(m->cap - 1);
    uint64_t h = mix64(key) & mask;
    while (m->used[h] && m->k[h] != key) h = (h + 1) & mask;
    if (!m->used[h]) return;
    m->used[h] = 0;
    m->size--;
    uint64_t j = h;
    for (;;) {
        j = (j + 1) & mask;
        if (!m->used[j]) return;
        const uint64_t home = mix64(m->k[j]) & mask;
        /* move j back to the hole h unless its home lies cyclically in (h, j] */
        const int keep = (h <= j) ? (home > h && home <= j) : (home > h || home <= j);
        if (keep) continue;
        m->used[h] = 1; m->k[h] = m->k[j]; m->v[h] = m->v[j];
        m->used[j] = 0;
        h = j;
    }
}

static int valid_window(int n, int interval) { return n > 0 && interval > 0 && interval % n == 0; }

/* Per-namespace raw list sizes of a whole-table load (namespace_idx -1 and out-of-range indices
 * each form their own group). */
static int64_t ns_group(int32_t ns_idx, int n_ns) { return (ns_idx >= 0 && ns_idx < n_ns) ? ns_idx : -1; }

/* ClusterFlowRuleManager.applyClusterFlowRule (ClusterFlowRuleManager.java:325-372) applied to every
 * namespace at once.  Valid rules (FlowRuleUtil.isValidRule: flowId > 0, count >= 0, window config)
 * are deduplicated by flowId: ruleMap.put keeps the last rule, the dense index is the first
 * position.  ClusterMetricStatistics.putMetricIfAbsent (CFRM:361-362) runs in list order, so a
 * flowId that already has a metric keeps it -- with its OLD sampleCount / windowIntervalMs and its
 * counters -- and a new flowId gets the window of its first occurrence.  A flowId that left the
 * table loses its metric (clearAndResetRulesConditional -> removeMetric, CFRM:285-301) unless its
 * namespace's new list is empty: clearAndResetRulesFor (CFRM:268-283) leaves METRIC_MAP alone, so
 * the metric stays, unreachable, and is picked up again if the flowId comes back.  nowCalls
 * (CurrentConcurrencyManager) survives only for flowIds present before and after (CFRM:356-358). */
int orc_engine_load_flow_rules(orc_engine *e, const orc_flow_rule *rules, int n) {
    /* raw list size per namespace group */
    int64_t *raw = (int64_t *)calloc((size_t)e->n_ns + 1, sizeof(int64_t));
    for (int i = 0; i < n; i++) raw[ns_group(rules[i].namespace_idx, e->n_ns) + 1]++;
    /* dense table */
    orc_flow_rule *nr = (orc_flow_rule *)calloc((size_t)(n > 0 ? n : 1), sizeof(orc_flow_rule));
    kvmap nidx;
    kv_init(&nidx);
    int nn = 0;
    for (int i = 0; i < n; i++) {
        const orc_flow_rule *r = &rules[i];
        if (r->flow_id <= 0 || !(r->count >= 0) || !valid_window(r->sample_count, r->window_interval_ms)) continue;
        int64_t *p = kv_find(&nidx, (uint64_t)r->flow_id);
        if (p) { nr[*p] = *r; continue; }
        *kv_insert(&nidx, (uint64_t)r->flow_id, 0) = nn;
        nr[nn++] = *r;
        /* putMetricIfAbsent with the first occurrence's window */
        if (!kv_find(&e->metric_map, (uint64_t)r->flow_id))
            *kv_insert(&e->metric_map, (uint64_t)r->flow_id, 0) =
                (int64_t)(intptr_t)orc_cm_new(r->sample_count, r->window_interval_ms);
    }
    /* flowIds that left: drop the metric unless their namespace's list is empty */
    for (int i = 0; i < e->n_rules; i++) {
        const orc_flow_rule *o = &e->rules[i];
        if (kv_find(&nidx, (uint64_t)o->flow_id)) continue;
        if (raw[ns_group(o->namespace_idx, e->n_ns) + 1] == 0) continue;          /* orphaned, kept */
        int64_t *m = kv_find(&e->metric_map, (uint64_t)o->flow_id);
        if (m) orc_cm_free((orc_cluster_metric *)(intptr_t)*m);
        kv_erase(&e->metric_map, (uint64_t)o->flow_id);
    }
    free(e->rules); free(e->cm);
    e->rules = nr;
    e->n_rules = nn;
    e->cm = (orc_cluster_metric **)calloc((size_t)(nn > 0 ? nn : 1), sizeof(orc_cluster_metric *));
    kvmap now;
    kv_init(&now);
    for (int i = 0; i < nn; i++) {
        e->cm[i] = (orc_cluster_metric *)(intptr_t)*kv_find(&e->metric_map, (uint64_t)nr[i].flow_id);
        const int64_t *old = kv_find(&e->now_calls, (uint64_t)nr[i].flow_id);
        *kv_insert(&now, (uint64_t)nr[i].flow_id, 0) = old ? *old : 0;
    }
    kv_free(&e->now_calls);
    e->now_calls = now;
    kv_free(&e->rule_by_fid);
    e->rule_by_fid = nidx;
    free(raw);
    return nn;
}

/* ClusterServerConfigManager.applyGlobalFlowConfig with a new (sampleCount, intervalMs)
 * (ClusterServerConfigManager.java:333-343): ClusterMetricStatistics.resetFlowMetrics and
 * ClusterParamMetricStatistics.resetFlowMetrics replace EVERY metric -- orphans included -- with a
 * fresh one of the server window. */
int orc_engine_reset_metrics(orc_engine *e, int sample_count, int interval_ms) {
    if (!valid_window(sample_count, interval_ms)) return -1;
    for (int64_t j = 0; j < e->metric_map.cap; j++) {
        if (!e->metric_map.used[j]) continue;
        orc_cm_free((orc_cluster_metric *)(intptr_t)e->metric_map.v[j]);
        e->metric_map.v[j] = (int64_t)(intptr_t)orc_cm_new(sample_count, interval_ms);
    }
    for (int i = 0; i < e->n_rules; i++)
        e->cm[i] = (orc_cluster_metric *)(intptr_t)*kv_find(&e->metric_map, (uint64_t)e->rules[i].flow_id);
    for (int64_t j = 0; j < e->param_metric_map.cap; j++) {
        if (!e->param_metric_map.used[j]) continue;
        orc_pm_free((orc_param_metric *)(intptr_t)e->param_metric_map.v[j]);
        e->param_metric_map.v[j] = (int64_t)(intptr_t)orc_pm_new(sample_count, interval_ms, 4000);
    }
    for (int i = 0; i < e->n_prules; i++)
        e->prules[i].pm = (orc_param_metric *)(intptr_t)*kv_find(&e->param_metric_map, (uint64_t)e->prules[i].r.flow_id);
    return 0;
}

/* Window of the metric behind dense flow index idx: {sampleCount, intervalMs}; -1 if none. */
int orc_engine_flow_window(const orc_engine *e, int32_t idx, int32_t *out2) {
    if (idx < 0 || idx >= e->n_rules || !e->cm[idx]) return -1;
    out2[0] = e->cm[idx]->la.n;
    out2[1] = e->cm[idx]->la.interval;
    return 0;
}

/* Number of metrics held (reachable + orphaned): METRIC_MAP.size(). */
int64_t orc_engine_metric_count(const orc_engine *e) { return e->metric_map.size; }

/* GRL:46-55 tryPass(namespace) */
static int engine_allow_proceed(orc_engine *e, int32_t ns, int64_t t) {
    if (ns < 0 || ns >= e->n_ns) return 0;          /* namespace == null -> false */
    if (!e->lim[ns]) return 1;                      /* no limiter -> true */
    return orc_limiter_try_pass(e->lim[ns], t);
}

/* CFC:38-48 calcGlobalThreshold */
static double calc_global_threshold(const orc_engine *e, const orc_flow_rule *r) {
    double count = r->count;
    if (r->threshold_type == 1) return count;
    int connected = (r->namespace_idx >= 0 && r->namespace_idx < e->n_ns) ? e->ns[r->namespace_idx].connected_count : 0;
    return count * (double)connected;
}

static void set_result(int8_t *st, int32_t *rem, int32_t *wait, int s, int32_t r, int32_t w) {
    *st = (int8_t)s;
    *rem = r;
    if (wait) *wait = w;
}

/* CFC:55-112 acquireClusterToken */
static void cluster_flow_check(orc_engine *e, int32_t idx, int32_t acquire, int prio, int64_t t,
                               int8_t *st, int32_t *rem, int32_t *wait) {
    const orc_flow_rule *r = &e->rules[idx];
    if (!engine_allow_proceed(e, r->namespace_idx, t)) { set_result(st, rem, wait, ORC_TOO_MANY_REQUEST, 0, 0); return; }
    orc_cluster_metric *m = e->cm[idx];
    if (!m) { set_result(st, rem, wait, ORC_FAIL, 0, 0); return; }
    double latest = orc_cm_get_avg(m, t, ORC_PASS);
    double global = calc_global_threshold(e, r) * e->cfg.exceed_count;
    double next = (global - latest) - (double)acquire;
    if (next >= 0) {
        orc_cm_add(m, t, ORC_PASS, acquire);
        orc_cm_add(m, t, ORC_PASS_REQUEST, 1);
        if (prio) orc_cm_add(m, t, ORC_OCCUPIED_PASS, acquire);
        set_result(st, rem, wait, ORC_OK, orc_java_d2i(next), 0);
        return;
    }
    if (prio) {
        double occupy_avg = orc_cm_get_avg(m, t, ORC_WAITING);
        if (occupy_avg <= e->cfg.max_occupy_ratio * global) {
            int w = orc_cm_try_occupy_next(m, t, ORC_PASS, acquire, global);
            if (w > 0) { set_result(st, rem, wait, ORC_SHOULD_WAIT, 0, w); return; }
        }
    }
    orc_cm_add(m, t, ORC_BLOCK, acquire);
    orc_cm_add(m, t, ORC_BLOCK_REQUEST, 1);
    if (prio) orc_cm_add(m, t, ORC_OCCUPIED_BLOCK, acquire);
    set_result(st, rem, wait, ORC_BLOCKED, 0, 0);
}

/* SCFC:33-65 (Envoy RLS): no limiter, no priority, threshold = count * exceedCount. */
static void simple_flow_check(orc_engine *e, int32_t idx, int32_t acquire, int64_t t,
                              int8_t *st, int32_t *rem, int32_t *wait) {
    const orc_flow_rule *r = &e->rules[idx];
    orc_cluster_metric *m = e->cm[idx];
    if (!m) { set_result(st, rem, wait, ORC_FAIL, 0, 0); return; }
    double latest = orc_cm_get_avg(m, t, ORC_PASS);
    double global = r->count * e->cfg.exceed_count;
    double next = (global - latest) - (double)acquire;
    if (next >= 0) {
        orc_cm_add(m, t, ORC_PASS, acquire);
        orc_cm_add(m, t, ORC_PASS_REQUEST, 1);
        set_result(st, rem, wait, ORC_OK, orc_java_d2i(next), 0);
    } else {
        orc_cm_add(m, t, ORC_BLOCK, acquire);
        orc_cm_add(m, t, ORC_BLOCK_REQUEST, 1);
        set_result(st, rem, wait, ORC_BLOCKED, 0, 0);
    }
}

/* DTS:37-48 requestToken (validation + rule lookup), then the rule's checker. */
void orc_request_token(orc_engine *e, int32_t idx, int32_t acquire, int prio, int64_t t,
                       int8_t *st, int32_t *rem, int32_t *wait) {
    if (idx == -2 || acquire <= 0) { set_result(st, rem, wait, ORC_BAD_REQUEST, 0, 0); return; }
    if (idx < 0 || idx >= e->n_rules) { set_result(st, rem, wait, ORC_NO_RULE_EXISTS, 0, 0); return; }
    if (e->rules[idx].checker == 1) simple_flow_check(e, idx, acquire, t, st, rem, wait);
    else cluster_flow_check(e, idx, acquire, prio, t, st, rem, wait);
}

void orc_flow_replay(orc_engine *e, int64_t n, const int32_t *flow_idx, const int32_t *acquire,
                     const uint8_t *flags, const int64_t *ts,
                     int8_t *status, int32_t *remaining, int32_t *wait_ms) {
    for (int64_t i = 0; i < n; i++)
        orc_request_token(e, flow_idx[i], acquire[i], flags ? (flags[i] & 1) : 0, ts[i],
                          &status[i], &remaining[i], wait_ms ? &wait_ms[i] : NULL);
}

/* Multi-threaded replay for the CPU baseline (BASELINE.md §2 mode ii): thread k owns the flows
 * with flow_idx mod T == k and processes their events in arrival order, so each flow still sees a
 * sequential replay.  Only valid without namespace limiters (they couple flows). */
typedef struct {
    orc_engine *e;
    int64_t n;
    const int32_t *flow_idx, *acquire;
    const uint8_t *flags;
    const int64_t *ts;
    int8_t *status;
    int32_t *remaining, *wait_ms;
    int T, k;
} mt_arg;

static void *mt_worker(void *p) {
    mt_arg *a = (mt_arg *)p;
    for (int64_t i = 0; i < a->n; i++) {
        const int32_t f = a->flow_idx[i];
        const int owner = f >= 0 ? (int)(f % a->T) : 0;
        if (owner != a->k) continue;
        orc_request_token(a->e, f, a->acquire[i], a->flags ? (a->flags[i] & 1) : 0, a->ts[i],
                          &a->status[i], &a->remaining[i], a->wait_ms ? &a->wait_ms[i] : NULL);
    }
    return NULL;
}

int orc_flow_replay_mt(orc_engine *e, int64_t n, const int32_t *flow_idx, const int32_t *acquire,
                       const uint8_t *flags, const int64_t *ts, int8_t *status, int32_t *remaining,
                       int32_t *wait_ms, int nthreads) {
    for (int i = 0; i < e->n_ns; i++)
        if (e->lim[i]) nthreads = 1;
    if (nthreads <= 1) {
        orc_flow_replay(e, n, flow_idx, acquire, flags, ts, status, remaining, wait_ms);
        return 1;
    }
    pthread_t th[256];
    mt_arg args[256];
    if (nthreads > 256) nthreads = 256;
    for (int k = 0; k < nthreads; k++) {
        args[k] = (mt_arg){e, n, flow_idx, acquire, flags, ts, status, remaining, wait_ms, nthreads, k};
        pthread_create(&th[k], NULL, mt_worker, &args[k]);
    }
    for (int k = 0; k < nthreads; k++) pthread_join(th[k], NULL);
    return nthreads;
}

int orc_engine_dump_flow(const orc_engine *e, int32_t idx, int64_t *out) {
    if (idx < 0 || idx >= e->n_rules || !e->cm[idx]) return -1;
    orc_cm_dump(e->cm[idx], out);
    return e->cm[idx]->la.n * (1 + ORC_NEVENTS) + ORC_NEVENTS + 1;
}

int64_t orc_engine_limiter_sum(orc_engine *e, int32_t ns, int64_t t) {
    if (ns < 0 || ns >= e->n_ns || !e->lim[ns]) return -1;
    return orc_limiter_get_sum(e->lim[ns], t);
}

/* ---- cluster hot-parameter path ---- */
/* ClusterParamFlowRuleManager.applyClusterParamRules (ClusterParamFlowRuleManager.java:318-360) for
 * every namespace at once, with the flow table's semantics: valid rules (ParamFlowRuleUtil.isValidRule:
 * count >= 0, window config, flowId > 0) deduplicated by flowId (last rule wins, first position keeps
 * the dense index); ClusterParamMetricStatistics.putMetricIfAbsent (:355-356) keeps the metric -- old
 * window and counters -- of a flowId present before and after; a flowId that left loses its metric
 * unless its namespace's list is empty (clearAndResetRulesFor keeps METRIC_MAP entries). */
int orc_engine_load_param_rules(orc_engine *e, const orc_param_rule *rules, int n,
                                const uint64_t *hot_keys, const int32_t *hot_counts, int n_hot) {
    int64_t *raw = (int64_t *)calloc((size_t)e->n_ns + 1, sizeof(int64_t));
    for (int i = 0; i < n; i++) raw[ns_group(rules[i].namespace_idx, e->n_ns) + 1]++;
    param_entry *np = (param_entry *)calloc((size_t)(n > 0 ? n : 1), sizeof(param_entry));
    kvmap nidx;
    kv_init(&nidx);
    int nn = 0;
    for (int i = 0; i < n; i++) {
        const orc_param_rule *r = &rules[i];
        if (r->flow_id <= 0 || !(r->count >= 0) || !valid_window(r->sample_count, r->window_interval_ms)) continue;
        int64_t *p = kv_find(&nidx, (uint64_t)r->flow_id);
        if (p) { np[*p].r = *r; continue; }
        *kv_insert(&nidx, (uint64_t)r->flow_id, 0) = nn;
        np[nn++].r = *r;
        if (!kv_find(&e->param_metric_map, (uint64_t)r->flow_id))
            *kv_insert(&e->param_metric_map, (uint64_t)r->flow_id, 0) =
                (int64_t)(intptr_t)orc_pm_new(r->sample_count, r->window_interval_ms, 4000);
    }
    for (int i = 0; i < e->n_prules; i++) {
        const orc_param_rule *o = &e->prules[i].r;
        if (kv_find(&nidx, (uint64_t)o->flow_id)) continue;
        if (raw[ns_group(o->namespace_idx, e->n_ns) + 1] == 0) continue;
        int64_t *m = kv_find(&e->param_metric_map, (uint64_t)o->flow_id);
        if (m) orc_pm_free((orc_param_metric *)(intptr_t)*m);
        kv_erase(&e->param_metric_map, (uint64_t)o->flow_id);
    }
    for (int i = 0; i < nn; i++)
        np[i].pm = (orc_param_metric *)(intptr_t)*kv_find(&e->param_metric_map, (uint64_t)np[i].r.flow_id);
    free(e->prules); free(e->hot_keys); free(e->hot_counts);
    e->prules = np;
    e->n_prules = nn;
    kv_free(&nidx);
    free(raw);
    e->n_hot = n_hot;
    e->hot_keys = (uint64_t *)calloc((size_t)(n_hot > 0 ? n_hot : 1), sizeof(uint64_t));
    e->hot_counts = (int32_t *)calloc((size_t)(n_hot > 0 ? n_hot : 1), sizeof(int32_t));
    if (n_hot > 0) {
        memcpy(e->hot_keys, hot_keys, sizeof(uint64_t) * (size_t)n_hot);
        memcpy(e->hot_counts, hot_counts, sizeof(int32_t) * (size_t)n_hot);
    }
    return nn;
}

/* getTopValues(number) of the param metric behind dense rule idx (ClusterParamMetric.java:84-127). */
int orc_engine_param_top_values(orc_engine *e, int32_t idx, int64_t t, int number, uint64_t *keys, double *avgs) {
    if (idx < 0 || idx >= e->n_prules || !e->prules[idx].pm) return 0;
    return orc_pm_top_values(e->prules[idx].pm, t, number, keys, avgs);
}

int orc_engine_param_window(const orc_engine *e, int32_t idx, int32_t *out2) {
    if (idx < 0 || idx >= e->n_prules || !e->prules[idx].pm) return -1;
    out2[0] = e->prules[idx].pm->la.n;
    out2[1] = e->prules[idx].pm->la.interval;
    return 0;
}

/* CPFC:101-120 calcGlobalThreshold(rule, value) */
/* ConnectionManager's connected count of a namespace changes (client PING / disconnect): every later
 * AVG_LOCAL threshold reads it (CFC:38-48, CPFC:101-111). */
void orc_engine_set_connected_count(orc_engine *e, int32_t ns, int32_t connected) {
    if (ns >= 0 && ns < e->n_ns) e->ns[ns].connected_count = connected;
}

static double param_threshold(const orc_engine *e, const orc_param_rule *r, uint64_t v) {
    double count = r->count;
    for (int i = 0; i < r->hot_n; i++)                       /* ParamFlowRule.java:157-162 */
        if (e->hot_keys[r->hot_begin + i] == v) { count = (double)e->hot_counts[r->hot_begin + i]; break; }
    if (r->threshold_type == 1) return count;
    int connected = (r->namespace_idx >= 0 && r->namespace_idx < e->n_ns) ? e->ns[r->namespace_idx].connected_count : 0;
    return count * (double)connected;
}

/* DTS:51-62 + CPFC:42-87 */
void orc_request_param_token(orc_engine *e, int32_t idx, int32_t acquire, int64_t t,
                             const uint64_t *values, int n_values, int8_t *st, int32_t *rem) {
    if (idx == -2 || acquire <= 0 || n_values <= 0) { *st = ORC_BAD_REQUEST; *rem = 0; return; }
    if (idx < 0 || idx >= e->n_prules) { *st = ORC_NO_RULE_EXISTS; *rem = 0; return; }
    const orc_param_rule *r = &e->prules[idx].r;
    if (t < 0 && r->namespace_idx >= 0 && r->namespace_idx < e->n_ns && e->lim[r->namespace_idx]) {
        /* RequestLimiter.tryPass at t < 0 (RL:81-87): the sum is 0, add(1) dies in currentWindow() == null
         * (LA:149-152) -> the engine's FAIL stand-in for the NullPointerException */
        *st = ORC_FAIL; *rem = 0; return;
    }
    if (!engine_allow_proceed(e, r->namespace_idx, t)) { *st = ORC_TOO_MANY_REQUEST; *rem = 0; return; }
    orc_param_metric *m = e->prules[idx].pm;
    if (!m) { *st = ORC_FAIL; *rem = 0; return; }
    if (t < 0) {
        /* LA:149-152 currentWindow(t < 0) == null, LA:375-378 values(t < 0) empty: every getAvg is 0, a
         * value with (T_v - 0) - a < 0 blocks the request untouched (CPFC:66-70); a request that passes
         * dies in addValue's currentWindow().value() (ClusterParamMetric.java:69, NullPointerException),
         * which the engine answers FAIL */
        for (int i = 0; i < n_values; i++)
            if ((param_threshold(e, r, values[i]) - 0.0) - (double)acquire < 0) { *st = ORC_BLOCKED; *rem = 0; return; }
        *st = ORC_FAIL; *rem = 0; return;
    }
    double remaining = -1;
    int passed = 1;
    for (int i = 0; i < n_values; i++) {
        double latest = orc_pm_get_avg(m, t, values[i]);
        double thr = param_threshold(e, r, values[i]);
        double next = (thr - latest) - (double)acquire;
        remaining = next;
        if (next < 0) { passed = 0; break; }
    }
    if (passed)
        for (int i = 0; i < n_values; i++) orc_pm_add_value(m, t, values[i], acquire);
    if (n_values > 1) remaining = -1;
    if (passed) { *st = ORC_OK; *rem = orc_java_d2i(remaining); }
    else { *st = ORC_BLOCKED; *rem = 0; }
}

void orc_param_replay(orc_engine *e, int64_t n, const int32_t *rule_idx, const int32_t *acquire,
                      const uint64_t *param_key, const int64_t *ts, int8_t *status, int32_t *remaining) {
    for (int64_t i = 0; i < n; i++)
        orc_request_param_token(e, rule_idx[i], acquire[i], ts[i], &param_key[i], 1, &status[i], &remaining[i]);
}

/* Rule-sharded multi-threaded param replay (CPU baseline only): thread k owns the
 * rules with rule_idx mod T == k (each rule's ClusterParamMetric is its own); without namespace
 * limiters (they couple rules) it is one thread. */
typedef struct {
    orc_engine *e;
    int64_t n;
    const int32_t *rule_idx, *acquire;
    const uint64_t *param_key;
    const int64_t *ts;
    int8_t *status;
    int32_t *remaining;
    int T, k;
} param_mt_arg;

static void *param_mt_worker(void *p) {
    param_mt_arg *a = (param_mt_arg *)p;
    for (int64_t i = 0; i < a->n; i++) {
        const int32_t r = a->rule_idx[i];
        if ((r >= 0 ? (int)(r % a->T) : 0) != a->k) continue;
        orc_request_param_token(a->e, r, a->acquire[i], a->ts[i], &a->param_key[i], 1, &a->status[i], &a->remaining[i]);
    }
    return NULL;
}

int orc_param_replay_mt(orc_engine *e, int64_t n, const int32_t *rule_idx, const int32_t *acquire,
                        const uint64_t *param_key, const int64_t *ts, int8_t *status, int32_t *remaining, int nthreads) {
    for (int i = 0; i < e->n_ns; i++)
        if (e->lim[i]) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    if (nthreads <= 1) {
        orc_param_replay(e, n, rule_idx, acquire, param_key, ts, status, remaining);
        return 1;
    }
    pthread_t th[256];
    param_mt_arg args[256];
    for (int k = 0; k < nthreads; k++) {
        args[k] = (param_mt_arg){e, n, rule_idx, acquire, param_key, ts, status, remaining, nthreads, k};
        pthread_create(&th[k], NULL, param_mt_worker, &args[k]);
    }
    for (int k = 0; k < nthreads; k++) pthread_join(th[k], NULL);
    return nthreads;
}

int64_t orc_engine_param_sum(orc_engine *e, int32_t idx, int64_t t, uint64_t key) {
    if (idx < 0 || idx >= e->n_prules || !e->prules[idx].pm) return 0;
    return orc_pm_get_sum(e->prules[idx].pm, t, key);
}

int orc_engine_param_overflowed(const orc_engine *e) {
    for (int i = 0; i < e->n_prules; i++)
        if (e->prules[i].pm && e->prules[i].pm->overflow) return 1;
    return 0;
}

/* ------------------------------------------------------------------ local StatisticNode */
/* SN:96-103: rollingCounterInSecond = ArrayMetric(SAMPLE_COUNT, INTERVAL) over an
 * OccupiableBucketLeapArray (occupy/OccupiableBucketLeapArray.java:29-101) whose borrowArray is a
 * FutureBucketLeapArray (occupy/FutureBucketLeapArray.java:28-53); rollingCounterInMinute =
 * ArrayMetric(60, 60000, false) over a plain BucketLeapArray. */
typedef struct {
    leap la;
    int64_t *c;          /* n x 6 MetricBucket counters */
    int64_t *minrt;      /* n MetricBucket.minRt (MB:38, reset to statisticMaxRt: MB:58-60) */
    int64_t scratch[ORC_M_NEVENTS];
    int64_t scratch_minrt;
    const int64_t *max_rt;   /* SentinelConfig.statisticMaxRt() of the node */
    int occupiable;      /* seed new / reset buckets from `borrow` (OBLA:40-64) */
    void *borrow;        /* bucket_array * (FutureBucketLeapArray) */
    int future;          /* FutureBucketLeapArray: deprecated iff time >= windowStart (FBLA:49-52) */
} bucket_array;

struct orc_stat_node {
    bucket_array sec, min, borrow;
    int occupy_timeout;  /* OccupyTimeoutProperty.occupyTimeout (default 500) */
    int64_t threads;     /* SN:108 curThreadNum (LongAdder) */
    int64_t max_rt;      /* SentinelConfig.statisticMaxRt (default 5000, SentinelConfig.java:63) */
};

static void ba_init(bucket_array *a, int n, int interval) {
    memset(a, 0, sizeof(*a));
    leap_init(&a->la, n, interval);
    a->c = (int64_t *)calloc((size_t)n * ORC_M_NEVENTS, sizeof(int64_t));
    a->minrt = (int64_t *)calloc((size_t)n, sizeof(int64_t));
}

static int ba_deprecated(const bucket_array *a, int64_t t, int i) {
    return a->future ? t >= a->la.start[i] : leap_deprecated(&a->la, t, i);
}

/* LA:290-303 getWindowValue(time): no roll; the bucket only if start <= time < start + win. */
static int64_t *ba_window_value(bucket_array *a, int64_t t) {
    if (t < 0) return NULL;
    int i = leap_idx(&a->la, t);
    if (!a->la.present[i]) return NULL;
    int64_t st = a->la.start[i];
    if (!(st <= t && t < st + a->la.win)) return NULL;   /* WindowWrap.isTimeInWindow (WW:93-95) */
    return a->c + (size_t)i * ORC_M_NEVENTS;
}

static int64_t *ba_current(bucket_array *a, int64_t t) {
    int i = 0;
    int act = leap_locate(&a->la, t, &i);
    if (act == LA_NULL) return NULL;
    if (act == LA_DETACHED) {
        memset(a->scratch, 0, sizeof(a->scratch));
        a->scratch_minrt = a->max_rt ? *a->max_rt : 0;
        return a->scratch;
    }
    int64_t *b = a->c + (size_t)i * ORC_M_NEVENTS;
    if ((act == LA_NEW || act == LA_RESET) && a->max_rt) a->minrt[i] = *a->max_rt;   /* initMinRt */
    if (act == LA_NEW) {
        memset(b, 0, sizeof(int64_t) * ORC_M_NEVENTS);
        if (a->occupiable) {                   /* OBLA:40-49 newEmptyBucket(time): reset(borrowBucket) */
            const int64_t *bb = ba_window_value((bucket_array *)a->borrow, t);
            if (bb) memcpy(b, bb, sizeof(int64_t) * ORC_M_NEVENTS);
        }
    } else if (act == LA_RESET) {
        memset(b, 0, sizeof(int64_t) * ORC_M_NEVENTS);
        if (a->occupiable) {                   /* OBLA:52-64 resetWindowTo: addPass((int) borrow.pass()) */
            const int64_t *bb = ba_window_value((bucket_array *)a->borrow, a->la.start[i]);
            if (bb) b[ORC_M_PASS] = (int32_t)bb[ORC_M_PASS];
        }
    }
    return b;
}

static int64_t ba_sum(bucket_array *a, int64_t t, int ev) {   /* ArrayMetric.pass()/block() */
    ba_current(a, t);
    int64_t s = 0;
    for (int i = 0; i < a->la.n; i++)
        if (a->la.present[i] && !ba_deprecated(a, t, i)) s = wrap_add64(s, a->c[(size_t)i * ORC_M_NEVENTS + ev]);
    return s;
}

static void ba_add(bucket_array *a, int64_t t, int ev, int64_t x) {
    int64_t *b = ba_current(a, t);
    if (b) b[ev] = wrap_add64(b[ev], x);
}

/* MetricBucket.addRT (MB:132-139) through ArrayMetric.addRT (AM:249-252): roll, add, keep the min. */
static void ba_add_rt(bucket_array *a, int64_t t, int64_t rt) {
    int64_t *b = ba_current(a, t);
    if (!b) return;
    b[ORC_M_RT] = wrap_add64(b[ORC_M_RT], rt);
    int64_t *m = b == a->scratch ? &a->scratch_minrt : &a->minrt[(b - a->c) / ORC_M_NEVENTS];
    if (rt < *m) *m = rt;
}

/* Read-only view of the windows as a roll at t would leave them (LA:316-318 after currentWindow):
 * buckets of the epochs > epoch(t) - n, future buckets included; the bucket the roll would reset
 * (epoch(t) - n, same slot) is not counted. */
static int ba_view_valid(const bucket_array *a, int64_t t, int i) {
    if (!a->la.present[i]) return 0;
    const int64_t E = t / a->la.win;
    return a->la.start[i] / a->la.win > E - a->la.n;
}

/* ArrayMetric.minRt (AM:142-153): max(1, min(statisticMaxRt, minRt of the valid buckets)). */
static int64_t ba_min_rt(const bucket_array *a, int64_t t, int64_t max_rt) {
    int64_t rt = max_rt;
    for (int i = 0; i < a->la.n; i++)
        if (ba_view_valid(a, t, i) && a->minrt[i] < rt) rt = a->minrt[i];
    return rt > 1 ? rt : 1;
}

static int64_t ba_view_sum(const bucket_array *a, int64_t t, int ev) {
    int64_t s = 0;
    for (int i = 0; i < a->la.n; i++)
        if (ba_view_valid(a, t, i)) s = wrap_add64(s, a->c[(size_t)i * ORC_M_NEVENTS + ev]);
    return s;
}

orc_stat_node *orc_node_new(int sample_count, int interval_ms) {
    orc_stat_node *nd = (orc_stat_node *)calloc(1, sizeof(*nd));
    nd->max_rt = 5000;
    ba_init(&nd->sec, sample_count, interval_ms);
    ba_init(&nd->borrow, sample_count, interval_ms);     /* OBLA:36 */
    nd->borrow.future = 1;
    nd->sec.occupiable = 1;
    nd->sec.borrow = &nd->borrow;
    ba_init(&nd->min, 60, 60 * 1000);
    nd->sec.max_rt = &nd->max_rt;
    nd->min.max_rt = &nd->max_rt;
    nd->occupy_timeout = 500;                            /* OccupyTimeoutProperty.java:40 */
    return nd;
}

void orc_node_set_max_rt(orc_stat_node *nd, int64_t ms) { nd->max_rt = ms; }

void orc_node_free(orc_stat_node *nd) {
    if (!nd) return;
    leap_free(&nd->sec.la); free(nd->sec.c); free(nd->sec.minrt);
    leap_free(&nd->borrow.la); free(nd->borrow.c); free(nd->borrow.minrt);
    leap_free(&nd->min.la); free(nd->min.c); free(nd->min.minrt);
    free(nd);
}

/* OccupyTimeoutProperty.updateTimeout (OTP:64-78): ignored when < 0 or > INTERVAL. */
void orc_node_set_occupy_timeout(orc_stat_node *nd, int ms) {
    if (ms < 0 || ms > nd->sec.la.interval) return;
    nd->occupy_timeout = ms;
}

int64_t orc_node_pass_sum(orc_stat_node *nd, int64_t t) { return ba_sum(&nd->sec, t, ORC_M_PASS); }
int64_t orc_node_block_sum(orc_stat_node *nd, int64_t t) { return ba_sum(&nd->sec, t, ORC_M_BLOCK); }
int64_t orc_node_total_pass(orc_stat_node *nd, int64_t t) { return ba_sum(&nd->min, t, ORC_M_PASS); }
int64_t orc_node_minute_block(orc_stat_node *nd, int64_t t) { return ba_sum(&nd->min, t, ORC_M_BLOCK); }
int64_t orc_node_minute_occupied(orc_stat_node *nd, int64_t t) { return ba_sum(&nd->min, t, ORC_M_OCCUPIED_PASS); }

/* ArrayMetric.waiting -> OBLA.currentWaiting (OBLA:66-76): roll the borrow array, sum the future buckets. */
int64_t orc_node_waiting(orc_stat_node *nd, int64_t t) { return ba_sum(&nd->borrow, t, ORC_M_PASS); }

double orc_node_pass_qps(orc_stat_node *nd, int64_t t) {          /* SN:200-202 */
    return (double)orc_node_pass_sum(nd, t) / nd->sec.la.interval_sec;
}

void orc_node_add_pass_request(orc_stat_node *nd, int64_t t, int count) {   /* SN:246-249 */
    ba_add(&nd->sec, t, ORC_M_PASS, count);
    ba_add(&nd->min, t, ORC_M_PASS, count);
}

void orc_node_increase_block_qps(orc_stat_node *nd, int64_t t, int count) { /* SN:261-264 */
    ba_add(&nd->sec, t, ORC_M_BLOCK, count);
    ba_add(&nd->min, t, ORC_M_BLOCK, count);
}

/* OBLA:78-82 addWaiting(time, n): borrowArray.currentWindow(time).add(PASS, n) */
void orc_node_add_waiting(orc_stat_node *nd, int64_t future_time, int count) {
    ba_add(&nd->borrow, future_time, ORC_M_PASS, count);
}

/* SN:333-336 addOccupiedPass: the MINUTE counter's OCCUPIED_PASS and PASS */
void orc_node_add_occupied_pass(orc_stat_node *nd, int64_t t, int count) {
    ba_add(&nd->min, t, ORC_M_OCCUPIED_PASS, count);
    ba_add(&nd->min, t, ORC_M_PASS, count);
}

/* SN:288-320 tryOccupyNext(currentTime, acquireCount, threshold); INTERVAL / SAMPLE_COUNT are the
 * node's own second-window configuration. */
int64_t orc_node_try_occupy_next(orc_stat_node *nd, int64_t t, int acquire, double threshold) {
    const int interval = nd->sec.la.interval;
    const double max_count = threshold * (double)interval / 1000;
    const int64_t current_borrow = orc_node_waiting(nd, t);
    if ((double)current_borrow >= max_count) return nd->occupy_timeout;
    const int wl = interval / nd->sec.la.n;
    int64_t earliest = t - t % wl + wl - interval;
    int idx = 0;
    int64_t current_pass = orc_node_pass_sum(nd, t);
    while (earliest < t) {
        const int64_t wait = (int64_t)idx * wl + wl - t % wl;
        if (wait >= nd->occupy_timeout) break;
        const int64_t *b = ba_window_value(&nd->sec, earliest);       /* ArrayMetric.getWindowPass */
        const int64_t window_pass = b ? b[ORC_M_PASS] : 0;
        const int64_t lhs = wrap_add64(wrap_add64(wrap_add64(current_pass, current_borrow), acquire), -window_pass);
        if ((double)lhs <= max_count) return wait;
        earliest += wl;
        current_pass = wrap_add64(current_pass, -window_pass);
        idx++;
    }
    return nd->occupy_timeout;
}

/* DC:49-76 (non-prioritized): curCount + acquireCount > count  -> block. int + int wraps. */
int orc_default_controller_can_pass(orc_stat_node *nd, double count, int grade, int acquire,
                                    int32_t cur_thread_num, int64_t t) {
    int32_t cur = grade == 0 ? cur_thread_num : orc_java_d2i(orc_node_pass_qps(nd, t));
    int32_t sum = (int32_t)((uint32_t)cur + (uint32_t)acquire);
    return !((double)sum > count);
}

int orc_default_controller_check(double node_value, double count, int grade, int acquire) {
    int32_t cur = grade == 0 ? (int32_t)node_value : orc_java_d2i(node_value);
    int32_t sum = (int32_t)((uint32_t)cur + (uint32_t)acquire);
    return !((double)sum > count);
}

/* One SphU.entry of a QPS-grade resource: DC:49-69 then StatisticSlot's booking (SS:55-116).
 * Returns 1 pass, 0 block; *wait = waitInMs of a prioritized pass (PriorityWaitException: the
 * entry passes after sleeping, only the thread count and the occupied / waiting counters move). */
int orc_local_entry(orc_stat_node *nd, double count, int acquire, int prioritized, int64_t t, int64_t *wait) {
    return orc_local_entry_ex(nd, count, 0.0, ORC_LR_QPS, acquire, prioritized, t, wait);
}

void orc_local_replay(orc_stat_node *nd, double count, int64_t n, const int32_t *acquire,
                      const int64_t *ts, uint8_t *out_pass) {
    for (int64_t i = 0; i < n; i++) {
        int64_t w;
        out_pass[i] = (uint8_t)orc_local_entry(nd, count, acquire[i], 0, ts[i], &w);
    }
}

void orc_local_replay_prio(orc_stat_node *nd, double count, int64_t n, const int32_t *acquire, const int64_t *ts,
                           const uint8_t *prio, uint8_t *out_pass, int64_t *out_wait) {
    for (int64_t i = 0; i < n; i++)
        out_pass[i] = (uint8_t)orc_local_entry(nd, count, acquire[i], prio ? (prio[i] & 1) : 0, ts[i], &out_wait[i]);
}

/* One SphU.entry of a resource with QPS and / or THREAD grade DefaultController rules
 * (FlowRuleChecker.checkFlow: rules in order, the first failure throws; DC:49-76):
 *   QPS    cur = (int) passQps      THREAD cur = (int) curThreadNum  (SN:241-243: long -> int cast)
 *   block iff (double)(cur + acquire) > count, int add wrapping; only a QPS rule's failure of a
 *   prioritized entry tries tryOccupyNext (PriorityWaitException: the remaining rules are skipped).
 * Every QPS rule must pass, so `qps_count` is the smallest QPS count (likewise `thread_count`);
 * flags: ORC_LR_QPS / ORC_LR_THREAD present, ORC_LR_THREAD_FIRST the THREAD rule precedes the QPS
 * one.  Then StatisticSlot.entry (SS:55-123): pass -> increaseThreadNum + addPassRequest, occupied
 * pass -> increaseThreadNum, block -> increaseBlockQps.  Returns 1 pass, 0 block. */
int orc_local_entry_ex(orc_stat_node *nd, double qps_count, double thread_count, int flags, int acquire,
                       int prioritized, int64_t t, int64_t *wait) {
    *wait = 0;
    const int has_q = flags & ORC_LR_QPS, has_t = flags & ORC_LR_THREAD;
    const int thread_first = (flags & ORC_LR_THREAD_FIRST) != 0;
    for (int pass = 0; pass < 2; pass++) {
        const int check_thread = thread_first ? pass == 0 : pass == 1;
        if (check_thread) {
            if (!has_t) continue;
            const int32_t cur = (int32_t)nd->threads;                                  /* SN:242 */
            const int32_t sum = (int32_t)((uint32_t)cur + (uint32_t)acquire);
            if ((double)sum > thread_count) goto blocked;
        } else {
            if (!has_q) continue;
            if (orc_default_controller_can_pass(nd, qps_count, 1, acquire, 0, t)) continue;
            if (prioritized) {                                                         /* DC:52-64 */
                const int64_t w = orc_node_try_occupy_next(nd, t, acquire, qps_count);
                if (w < nd->occupy_timeout) {
                    orc_node_add_waiting(nd, t + w, acquire);
                    orc_node_add_occupied_pass(nd, t, acquire);
                    *wait = w;
                    nd->threads = wrap_add64(nd->threads, 1);                          /* SS:81-82 */
                    return 1;
                }
            }
            goto blocked;
        }
    }
    nd->threads = wrap_add64(nd->threads, 1);                                          /* SS:62-63 */
    orc_node_add_pass_request(nd, t, acquire);
    return 1;
blocked:
    orc_node_increase_block_qps(nd, t, acquire);                                       /* SS:96-104 */
    return 0;
}

/* Entry.exit of an entry that passed (StatisticSlot.exit, SS:126-164; blocked entries book nothing):
 * at completeStatTime t, recordCompleteFor -> addRtAndSuccess(rt, count) (SN:252-258: SUCCESS and
 * RT into both windows, minRt kept per bucket), decreaseThreadNum, and increaseExceptionQps(count)
 * when the entry carries a business exception (Tracer.trace -> Entry.setError). */
void orc_local_exit(orc_stat_node *nd, int count, int64_t rt, int error, int64_t t) {
    ba_add(&nd->sec, t, ORC_M_SUCCESS, count);
    ba_add_rt(&nd->sec, t, rt);
    ba_add(&nd->min, t, ORC_M_SUCCESS, count);
    ba_add_rt(&nd->min, t, rt);
    nd->threads = wrap_add64(nd->threads, -1);
    if (error) {
        ba_add(&nd->sec, t, ORC_M_EXCEPTION, count);
        ba_add(&nd->min, t, ORC_M_EXCEPTION, count);
    }
}

/* Read-only view at t (the valid buckets, no roll): out[0..5] second window {PASS, BLOCK,
 * EXCEPTION, SUCCESS, RT, minRt}, out[6..12] minute window {PASS, BLOCK, OCCUPIED_PASS, EXCEPTION,
 * SUCCESS, RT, minRt}, out[13] curThreadNum. */
void orc_node_metrics(const orc_stat_node *nd, int64_t t, int64_t *out) {
    const int ev6[5] = {ORC_M_PASS, ORC_M_BLOCK, ORC_M_EXCEPTION, ORC_M_SUCCESS, ORC_M_RT};
    for (int k = 0; k < 5; k++) out[k] = ba_view_sum(&nd->sec, t, ev6[k]);
    out[5] = ba_min_rt(&nd->sec, t, nd->max_rt);
    const int ev7[6] = {ORC_M_PASS, ORC_M_BLOCK, ORC_M_OCCUPIED_PASS, ORC_M_EXCEPTION, ORC_M_SUCCESS, ORC_M_RT};
    for (int k = 0; k < 6; k++) out[6 + k] = ba_view_sum(&nd->min, t, ev7[k]);
    out[12] = ba_min_rt(&nd->min, t, nd->max_rt);
    out[13] = nd->threads;
}

/* OccupiableBucketLeapArray surface for the reference's own tests (OccupiableBucketLeapArrayTest). */
int64_t orc_node_sec_window_pass(orc_stat_node *nd, int64_t t) {     /* currentWindow(t).value().pass() */
    int64_t *b = ba_current(&nd->sec, t);
    return b ? b[ORC_M_PASS] : 0;
}
void orc_node_sec_window_add_pass(orc_stat_node *nd, int64_t t, int n) { ba_add(&nd->sec, t, ORC_M_PASS, n); }
/* values(t) without a roll: {count of buckets, sum of PASS} */
int64_t orc_node_sec_values(orc_stat_node *nd, int64_t t, int64_t *sum) {
    int64_t k = 0, s = 0;
    for (int i = 0; i < nd->sec.la.n; i++)
        if (nd->sec.la.present[i] && !ba_deprecated(&nd->sec, t, i)) { k++; s = wrap_add64(s, nd->sec.c[(size_t)i * ORC_M_NEVENTS]); }
    *sum = s;
    return k;
}

/* ------------------------------------------------------------------ local rule graph (a9) */
/* FlowRuleChecker with every limitApp / strategy (FRC:44-145) over the node graph the slot chain
 * builds: a ClusterNode per resource (created by its first entry, ClusterBuilderSlot.java:74-92), an
 * origin StatisticNode per (resource, origin) (ClusterNode.getOrCreateOriginNode, set when the
 * context's origin is non-empty: CBS:97-100), a DefaultNode per (context, resource) whose
 * increaseThreadNum / addPassRequest / increaseBlockQps / addRtAndSuccess / decreaseThreadNum /
 * increaseExceptionQps also reach the ClusterNode (DefaultNode.java:110-143).  Rules of a resource
 * are checked in list order after FlowRuleUtil.buildFlowRuleMap's stable FlowRuleComparator sort
 * (non-"default" limitApps first, FlowRuleComparator.java:30-55; the caller passes FlowRuleManager's
 * order), invalid ones dropped (FlowRuleUtil.isValidRule:167-238). */
struct orc_lgraph {
    int n_res, n_on, n_dn;
    orc_stat_node **cn, **on, **dn;
    uint8_t *created;          /* ClusterNode exists (ClusterBuilderSlot.clusterNodeMap) */
    int32_t *roff;             /* rules of resource r: rules[roff[r] .. roff[r + 1]) */
    orc_local_rule *rules;
};

static int lrule_valid(const orc_local_rule *r, int n_res) {
    if (r->resource < 0 || r->resource >= n_res || !(r->count >= 0) || r->strategy < 0) return 0;  /* FRU:168-169 */
    if (r->grade == 1) {                                       /* QPS: checkStrategyField (FRU:233-238) */
        if (r->strategy > 2) return 1;                         /* unknown strategy: valid, selects no node */
        return r->strategy == 0 || r->ref >= 0;
    }
    return r->grade == 0;                                      /* THREAD: checkClusterConcurrentField only */
}

orc_lgraph *orc_lgraph_new(const orc_local_rule *rules, int n, int n_res, int n_origin_nodes, int n_default_nodes,
                           int sample_count, int interval_ms) {
    orc_lgraph *g = (orc_lgraph *)calloc(1, sizeof(*g));
    g->n_res = n_res; g->n_on = n_origin_nodes; g->n_dn = n_default_nodes;
    g->cn = (orc_stat_node **)calloc((size_t)(n_res > 0 ? n_res : 1), sizeof(void *));
    g->on = (orc_stat_node **)calloc((size_t)(n_origin_nodes > 0 ? n_origin_nodes : 1), sizeof(void *));
    g->dn = (orc_stat_node **)calloc((size_t)(n_default_nodes > 0 ? n_default_nodes : 1), sizeof(void *));
    for (int i = 0; i < n_res; i++) g->cn[i] = orc_node_new(sample_count, interval_ms);
    for (int i = 0; i < n_origin_nodes; i++) g->on[i] = orc_node_new(sample_count, interval_ms);
    for (int i = 0; i < n_default_nodes; i++) g->dn[i] = orc_node_new(sample_count, interval_ms);
    g->created = (uint8_t *)calloc((size_t)(n_res > 0 ? n_res : 1), 1);
    g->roff = (int32_t *)calloc((size_t)n_res + 1, sizeof(int32_t));
    g->rules = (orc_local_rule *)calloc((size_t)(n > 0 ? n : 1), sizeof(orc_local_rule));
    /* per resource: valid rules in the given order, duplicates dropped (the HashSet), then the stable
     * comparator sort: every non-"default" limitApp before the "default" ones */
    int k = 0;
    for (int r = 0; r < n_res; r++) {
        g->roff[r] = k;
        for (int pass = 0; pass < 2; pass++)
            for (int i = 0; i < n; i++) {
                const orc_local_rule *x = &rules[i];
                if (x->resource != r || !lrule_valid(x, n_res)) continue;
                const int lim = x->limit_app < 0 ? ORC_LIMIT_APP_DEFAULT : x->limit_app;   /* blank -> default */
                if ((lim == ORC_LIMIT_APP_DEFAULT) != (pass == 1)) continue;
                int dup = 0;
                for (int j = g->roff[r]; j < k && !dup; j++)
                    dup = g->rules[j].grade == x->grade && g->rules[j].count == x->count &&
                          g->rules[j].strategy == x->strategy && g->rules[j].limit_app == lim && g->rules[j].ref == x->ref;
                if (dup) continue;
                g->rules[k] = *x;
                g->rules[k].limit_app = lim;
                k++;
            }
    }
    g->roff[n_res] = k;
    return g;
}

void orc_lgraph_free(orc_lgraph *g) {
    if (!g) return;
    for (int i = 0; i < g->n_res; i++) orc_node_free(g->cn[i]);
    for (int i = 0; i < g->n_on; i++) orc_node_free(g->on[i]);
    for (int i = 0; i < g->n_dn; i++) orc_node_free(g->dn[i]);
    free(g->cn); free(g->on); free(g->dn); free(g->created); free(g->roff); free(g->rules); free(g);
}

void orc_lgraph_set_occupy_timeout(orc_lgraph *g, int ms) {
    for (int i = 0; i < g->n_res; i++) orc_node_set_occupy_timeout(g->cn[i], ms);
    for (int i = 0; i < g->n_on; i++) orc_node_set_occupy_timeout(g->on[i], ms);
    for (int i = 0; i < g->n_dn; i++) orc_node_set_occupy_timeout(g->dn[i], ms);
}

int orc_lgraph_n_rules(const orc_lgraph *g, int res) { return g->roff[res + 1] - g->roff[res]; }

/* FlowRuleManager.isOtherOrigin (FlowRuleManager.java:113-129) */
static int lgraph_other_origin(const orc_lgraph *g, int res, int origin) {
    if (origin < 0) return 0;                                  /* StringUtil.isEmpty(origin) */
    for (int j = g->roff[res]; j < g->roff[res + 1]; j++)
        if (g->rules[j].limit_app == origin) return 0;
    return 1;
}

/* FRC:87-103 selectReferenceNode */
static orc_stat_node *lgraph_ref_node(const orc_lgraph *g, const orc_local_rule *r, const orc_local_ctx *c) {
    if (r->ref < 0) return NULL;                               /* StringUtil.isEmpty(refResource) */
    if (r->strategy == ORC_STRATEGY_RELATE)                    /* ClusterBuilderSlot.getClusterNode(ref) */
        return r->ref < g->n_res && g->created[r->ref] ? g->cn[r->ref] : NULL;
    if (r->strategy == ORC_STRATEGY_CHAIN) return r->ref == c->context ? g->dn[c->default_node] : NULL;
    return NULL;
}

/* FRC:110-145 selectNodeByRequesterAndStrategy; filterOrigin: the origin is neither "default" nor
 * "other" (the interned ids 0 and 1) */
static orc_stat_node *lgraph_select(const orc_lgraph *g, int res, const orc_local_rule *r, const orc_local_ctx *c) {
    const int origin = c->origin;
    orc_stat_node *onode = origin >= 0 ? g->on[c->origin_node] : NULL;
    if (r->limit_app == origin && origin >= 2) {
        if (r->strategy == ORC_STRATEGY_DIRECT) return onode;
        return lgraph_ref_node(g, r, c);
    } else if (r->limit_app == ORC_LIMIT_APP_DEFAULT) {
        if (r->strategy == ORC_STRATEGY_DIRECT) return g->cn[res];
        return lgraph_ref_node(g, r, c);
    } else if (r->limit_app == ORC_LIMIT_APP_OTHER && lgraph_other_origin(g, res, origin)) {
        if (r->strategy == ORC_STRATEGY_DIRECT) return onode;
        return lgraph_ref_node(g, r, c);
    }
    return NULL;
}

/* One SphU.entry(resource) in context c: ClusterBuilderSlot (node creation), FlowSlot (every rule in
 * order, DefaultController.canPass on the selected node, DC:49-69), StatisticSlot.entry's booking on
 * the DefaultNode (+ ClusterNode) and the origin node (SS:55-116).  1 pass, 0 block; *wait as
 * orc_local_entry_ex. */
int orc_lgraph_entry(orc_lgraph *g, int res, int acquire, int prioritized, int64_t t, const orc_local_ctx *c,
                     int64_t *wait) {
    *wait = 0;
    g->created[res] = 1;
    orc_stat_node *dn = g->dn[c->default_node], *cn = g->cn[res];
    orc_stat_node *on = c->origin >= 0 ? g->on[c->origin_node] : NULL;
    int blocked = 0, occupied = 0;
    for (int j = g->roff[res]; j < g->roff[res + 1] && !blocked && !occupied; j++) {
        const orc_local_rule *r = &g->rules[j];
        orc_stat_node *nd = lgraph_select(g, res, r, c);
        if (!nd) continue;                                     /* FRC:78-81 no node -> pass */
        const int32_t cur = r->grade == 0 ? (int32_t)nd->threads : orc_java_d2i(orc_node_pass_qps(nd, t));
        if (!((double)(int32_t)((uint32_t)cur + (uint32_t)acquire) > r->count)) continue;
        if (prioritized && r->grade == 1) {                    /* DC:52-64 */
            const int64_t w = orc_node_try_occupy_next(nd, t, acquire, r->count);
            if (w < nd->occupy_timeout) {
                orc_node_add_waiting(nd, t + w, acquire);
                orc_node_add_occupied_pass(nd, t, acquire);
                *wait = w;
                occupied = 1;                                  /* PriorityWaitException */
                continue;
            }
        }
        blocked = 1;
    }
    if (blocked) {                                             /* SS:96-104 */
        orc_node_increase_block_qps(dn, t, acquire);
        orc_node_increase_block_qps(cn, t, acquire);
        if (on) orc_node_increase_block_qps(on, t, acquire);
        return 0;
    }
    dn->threads = wrap_add64(dn->threads, 1);                  /* SS:62-69 / 81-86 */
    cn->threads = wrap_add64(cn->threads, 1);
    if (!occupied) {
        orc_node_add_pass_request(dn, t, acquire);
        orc_node_add_pass_request(cn, t, acquire);
    }
    if (on) {
        on->threads = wrap_add64(on->threads, 1);
        if (!occupied) orc_node_add_pass_request(on, t, acquire);
    }
    return 1;
}

/* Entry.exit of a passed entry (SS:126-164): recordCompleteFor(DefaultNode) -- which also books the
 * ClusterNode -- then recordCompleteFor(origin node). */
void orc_lgraph_exit(orc_lgraph *g, int res, int count, int64_t rt, int error, int64_t t, const orc_local_ctx *c) {
    orc_local_exit(g->dn[c->default_node], count, rt, error, t);
    orc_local_exit(g->cn[res], count, rt, error, t);
    if (c->origin >= 0) orc_local_exit(g->on[c->origin_node], count, rt, error, t);
}

/* Arrival-order replay of a batch (flags: bit 0 prioritized, bit 1 exit, bit 2 error); status OK /
 * BLOCKED, NO_RULE_EXISTS for an unknown resource or node index, FAIL for t < 0 (as the GPU path). */
void orc_lgraph_replay(orc_lgraph *g, int64_t n, const int32_t *res, const int32_t *acquire, const int64_t *ts,
                       const orc_local_ctx *ctx, const uint8_t *flags, const int64_t *rt, int8_t *status,
                       int32_t *wait) {
    for (int64_t i = 0; i < n; i++) {
        const orc_local_ctx *c = &ctx[i];
        wait[i] = 0;
        if (res[i] < 0 || res[i] >= g->n_res || c->default_node < 0 || c->default_node >= g->n_dn ||
            (c->origin >= 0 && (c->origin_node < 0 || c->origin_node >= g->n_on))) { status[i] = 3; continue; }
        if (ts[i] < 0) { status[i] = -1; continue; }
        const uint8_t f = flags ? flags[i] : 0;
        if (f & 2) {
            orc_lgraph_exit(g, res[i], acquire[i], rt ? rt[i] : 0, (f & 4) != 0, ts[i], c);
            status[i] = 0;
            continue;
        }
        int64_t w;
        status[i] = orc_lgraph_entry(g, res[i], acquire[i], f & 1, ts[i], c, &w) ? 0 : 1;
        wait[i] = (int32_t)w;
    }
}

/* orc_node_metrics of node `idx` of kind 0 ClusterNode, 1 origin node, 2 DefaultNode */
int orc_lgraph_node_metrics(orc_lgraph *g, int kind, int idx, int64_t t, int64_t *out14) {
    orc_stat_node *nd = NULL;
    if (kind == 0 && idx >= 0 && idx < g->n_res) nd = g->cn[idx];
    if (kind == 1 && idx >= 0 && idx < g->n_on) nd = g->on[idx];
    if (kind == 2 && idx >= 0 && idx < g->n_dn) nd = g->dn[idx];
    if (!nd) return -1;
    orc_node_metrics(nd, t, out14);
    return 0;
}

/* ------------------------------------------------------------------ local param token bucket */
/* PFC:127-202 passDefaultLocalCheck, single-threaded (every CAS succeeds). The two CacheMaps are
 * ParameterMetric's ruleTokenCounter / ruleTimeCounter (ParameterMetric.java:95-118); LRU
 * eviction is not restated (exact parity only below the capacity). */
struct orc_param_bucket {
    kvmap time_ctr;
    kvmap token_ctr;
};

orc_param_bucket *orc_pbucket_new(void) {
    orc_param_bucket *b = (orc_param_bucket *)calloc(1, sizeof(*b));
    kv_init(&b->time_ctr);
    kv_init(&b->token_ctr);
    return b;
}

void orc_pbucket_free(orc_param_bucket *b) {
    if (!b) return;
    kv_free(&b->time_ctr);
    kv_free(&b->token_ctr);
    free(b);
}

int orc_pbucket_pass_default(orc_param_bucket *b, uint64_t key, int64_t token_count, int64_t burst,
                             int64_t duration_sec, int acquire, int64_t t) {
    if (token_count == 0) return 0;                                   /* PFC:143-145 */
    int64_t max_count = wrap_add64(token_count, burst);               /* PFC:147 */
    if ((int64_t)acquire > max_count) return 0;                       /* PFC:148-150 */
    int64_t *last = kv_find(&b->time_ctr, key);
    if (!last) {                                                      /* PFC:155-160 */
        kv_insert(&b->time_ctr, key, t);
        if (!kv_find(&b->token_ctr, key)) kv_insert(&b->token_ctr, key, max_count - acquire);
        return 1;
    }
    int64_t pass_time = t - *last;                                    /* PFC:163 */
    int64_t dur_ms = wrap_mul64(duration_sec, 1000);
    if (pass_time > dur_ms) {                                         /* PFC:165 */
        int64_t *old = kv_find(&b->token_ctr, key);
        if (!old) {
            kv_insert(&b->token_ctr, key, max_count - acquire);
            *kv_find(&b->time_ctr, key) = t;
            return 1;
        }
        int64_t rest = *old;
        int64_t to_add = wrap_mul64(pass_time, token_count) / dur_ms;  /* long arithmetic, wraps */
        int64_t new_qps = wrap_add64(to_add, rest) > max_count ? (max_count - acquire)
                                                               : wrap_add64(rest, to_add) - acquire;
        if (new_qps < 0) return 0;
        *old = new_qps;
        *kv_find(&b->time_ctr, key) = t;
        return 1;
    }
    int64_t *old = kv_find(&b->token_ctr, key);                       /* PFC:186-198 */
    if (old) {
        if (*old - acquire >= 0) { *old -= acquire; return 1; }
        return 0;
    }
    return -1;   /* time counter present, token counter absent: only after LRU eviction (unpinned) */
}

/* ------------------------------------------------------------------ multi-value cluster params */
/* A batch of requestParamToken calls with value lists, in arrival order (CPFC:42-87 per call). */
void orc_param_multi_replay(orc_engine *e, int64_t n, const int32_t *rule_idx, const int32_t *acquire,
                            const int64_t *ts, const int32_t *vbegin, const int32_t *vcount,
                            const uint64_t *values, int64_t n_values, int8_t *status, int32_t *remaining) {
    for (int64_t i = 0; i < n; i++) {
        const int32_t b = vbegin[i], c = vcount[i];
        if (c < 0 || b < 0 || (int64_t)b + c > n_values) { status[i] = ORC_BAD_REQUEST; remaining[i] = 0; continue; }
        orc_request_param_token(e, rule_idx[i], acquire[i], ts[i], values + b, c, &status[i], &remaining[i]);
    }
}

/* Audit of count-min verdicts against exact counters on the same history: replays the sequence
 * of decisions the sketch made (passes add to the exact ClusterParamMetric, blocks do not) and
 * counts (a) passes the exact checker would have blocked -- must be 0 for a one-sided sketch --
 * and (b) blocks the exact checker would have passed (false blocks). */
void orc_param_cm_audit(orc_engine *e, int64_t n, const int32_t *rule_idx, const int32_t *acquire,
                        const int64_t *ts, const int32_t *vbegin, const int32_t *vcount, const uint64_t *values,
                        const int8_t *status_cm, int64_t *violations, int64_t *false_blocks, int64_t *decided) {
    *violations = *false_blocks = *decided = 0;
    for (int64_t i = 0; i < n; i++) {
        if (status_cm[i] != ORC_OK && status_cm[i] != ORC_BLOCKED) continue;
        const int32_t idx = rule_idx[i];
        if (idx < 0 || idx >= e->n_prules || !e->prules[idx].pm) continue;
        const orc_param_rule *r = &e->prules[idx].r;
        orc_param_metric *m = e->prules[idx].pm;
        const uint64_t *v = values + vbegin[i];
        int exact_pass = 1;
        for (int j = 0; j < vcount[i]; j++) {
            double next = (param_threshold(e, r, v[j]) - orc_pm_get_avg(m, ts[i], v[j])) - (double)acquire[i];
            if (next < 0) { exact_pass = 0; break; }
        }
        (*decided)++;
        if (status_cm[i] == ORC_OK) {
            if (!exact_pass) (*violations)++;
            for (int j = 0; j < vcount[i]; j++) orc_pm_add_value(m, ts[i], v[j], acquire[i]);
        } else if (exact_pass) {
            (*false_blocks)++;
        }
    }
}

/* ------------------------------------------------------------------ local param engine */
/* ParamFlowChecker.passLocalCheck (PFC:78-103) with one ParameterMetric token/time counter pair
 * per rule (ParameterMetric.java:95-118); rules failing ParamFlowRuleUtil.isValidRule
 * (ParamFlowRuleUtil.java:46-52) are not loaded. */
typedef struct {
    orc_local_param_rule r;
    int valid;
    int64_t token_count;      /* (long) rule.count (PFC:139) */
    orc_param_bucket *b;
    kvmap hot;                /* param key -> hot-item count (PFC:138-142) */
    int grade;                /* RuleConstant.FLOW_GRADE_QPS (1, default) or FLOW_GRADE_THREAD (0) */
    kvmap threads;            /* ParameterMetric.threadCountMap entry of the rule's param index: key -> count */
} local_entry;

struct orc_local_engine {
    local_entry *rules;
    int n;
};

orc_local_engine *orc_lparam_new(const orc_local_param_rule *rules, int n, const uint64_t *hot_keys,
                                const int32_t *hot_counts, int n_hot) {
    orc_local_engine *e = (orc_local_engine *)calloc(1, sizeof(*e));
    e->n = n;
    e->rules = (local_entry *)calloc((size_t)(n > 0 ? n : 1), sizeof(local_entry));
    for (int i = 0; i < n; i++) {
        local_entry *le = &e->rules[i];
        le->r = rules[i];
        le->valid = rules[i].count >= 0 && rules[i].burst_count >= 0 && rules[i].duration_in_sec > 0;
        le->token_count = orc_java_d2l(rules[i].count);
        le->b = orc_pbucket_new();
        le->grade = 1;
        kv_init(&le->threads);
        kv_init(&le->hot);
        for (int h = 0; h < rules[i].hot_n; h++) {
            const int j = rules[i].hot_begin + h;
            if (j >= 0 && j < n_hot) *kv_insert(&le->hot, hot_keys[j], 0) = hot_counts[j];
        }
    }
    return e;
}

void orc_lparam_free(orc_local_engine *e) {
    if (!e) return;
    for (int i = 0; i < e->n; i++) {
        orc_pbucket_free(e->rules[i].b);
        kv_free(&e->rules[i].hot);
        kv_free(&e->rules[i].threads);
    }
    free(e->rules);
    free(e);
}

void orc_lparam_set_grades(orc_local_engine *e, const int32_t *grade, int n) {
    for (int i = 0; i < n && i < e->n; i++) e->rules[i].grade = grade[i];
}

/* THREAD grade (PFC:112-122): each value passes iff ++threadCount <= threshold (hot-item count, else
 * (long) rule.count), threadCount = ParameterMetric.getThreadCount (PM:241-249, absent 0); the
 * check reads, the entry callback writes: a passing check adds one per value
 * (ParamFlowStatisticEntryCallback -> PM.addThreadCount, PM:184-239; a repeated value twice). */
static int lparam_thread_check(local_entry *le, const uint64_t *vals, int32_t c) {
    for (int j = 0; j < c; j++) {
        const int64_t *hv = kv_find(&le->hot, vals[j]);
        const int64_t thr = hv ? *hv : le->token_count;
        const int64_t *tc = kv_find(&le->threads, vals[j]);
        const int64_t cur = tc ? *tc : 0;
        if (!(cur + 1 <= thr)) return 0;
    }
    for (int j = 0; j < c; j++) {
        int64_t *tc = kv_find(&le->threads, vals[j]);
        if (tc) *tc = (int32_t)((uint32_t)*tc + 1u);                 /* AtomicInteger.incrementAndGet */
        else kv_insert(&le->threads, vals[j], 1);
    }
    return 1;
}

/* Entry.exit -> ParamFlowStatisticExitCallback -> PM.decreaseThreadCount (PM:125-181): an absent
 * value gets a 0 entry (putIfAbsent), a present one is decremented and removed at <= 0. */
static void lparam_thread_exit(local_entry *le, const uint64_t *vals, int32_t c) {
    for (int j = 0; j < c; j++) {
        int64_t *tc = kv_find(&le->threads, vals[j]);
        if (!tc) { kv_insert(&le->threads, vals[j], 0); continue; }
        const int32_t v = (int32_t)((uint32_t)*tc - 1u);
        if (v <= 0) kv_erase(&le->threads, vals[j]);
        else *tc = v;
    }
}

int orc_lparam_thread_count(orc_local_engine *e, int32_t idx, uint64_t key) {
    if (idx < 0 || idx >= e->n) return -1;
    const int64_t *tc = kv_find(&e->rules[idx].threads, key);
    return tc ? (int)*tc : -1;
}

void orc_lparam_replay_ex(orc_local_engine *e, int64_t n, const int32_t *rule_idx, const int32_t *acquire,
                          const int64_t *ts, const int32_t *vbegin, const int32_t *vcount, const uint64_t *values,
                          int64_t n_values, const uint8_t *kinds, int8_t *status) {
    for (int64_t i = 0; i < n; i++) {
        const int32_t b = vbegin[i], c = vcount[i];
        if (c < 0 || b < 0 || (int64_t)b + c > n_values) { status[i] = ORC_BAD_REQUEST; continue; }
        const int32_t idx = rule_idx[i];
        if (idx < 0 || idx >= e->n || !e->rules[idx].valid) { status[i] = ORC_NO_RULE_EXISTS; continue; }
        local_entry *le = &e->rules[idx];
        if (kinds && kinds[i] == 1) {                    /* exit */
            if (le->grade == 0) lparam_thread_exit(le, values + b, c);
            status[i] = ORC_OK;
            continue;
        }
        if (c == 0) { status[i] = ORC_OK; continue; }
        if (le->grade == 0) { status[i] = lparam_thread_check(le, values + b, c) ? ORC_OK : ORC_BLOCKED; continue; }
        int st = ORC_OK;
        for (int j = 0; j < c; j++) {      /* every element must pass, no rollback (PFC:81-94) */
            const uint64_t key = values[b + j];
            const int64_t *hv = kv_find(&le->hot, key);
            const int64_t tok = hv ? *hv : le->token_count;
            const int r = orc_pbucket_pass_default(le->b, key, tok, le->r.burst_count, le->r.duration_in_sec,
                                                   acquire[i], ts[i]);
            if (r == 0) { st = ORC_BLOCKED; break; }
            if (r < 0) { st = ORC_FAIL; break; }
        }
        status[i] = (int8_t)st;
    }
}

void orc_lparam_replay(orc_local_engine *e, int64_t n, const int32_t *rule_idx, const int32_t *acquire,
                      const int64_t *ts, const int32_t *vbegin, const int32_t *vcount, const uint64_t *values,
                      int64_t n_values, int8_t *status) {
    orc_lparam_replay_ex(e, n, rule_idx, acquire, ts, vbegin, vcount, values, n_values, NULL, status);
}

int orc_lparam_state(orc_local_engine *e, int32_t idx, uint64_t key, int64_t *last, int64_t *tokens) {
    *last = *tokens = -1;
    if (idx < 0 || idx >= e->n) return 0;
    int64_t *l = kv_find(&e->rules[idx].b->time_ctr, key);
    int64_t *t = kv_find(&e->rules[idx].b->token_ctr, key);
    if (l) *last = *l;
    if (t) *tokens = *t;
    return l != NULL;
}

/* ------------------------------------------------------------------ concurrency tokens */
/* ConcurrentClusterFlowChecker (CCFC:35-101) replayed sequentially.  new_ids[i] is the token id an
 * acquire receives when it passes (the reference draws it from UUID.randomUUID()). */
static double conc_threshold(const orc_engine *e, const orc_flow_rule *r) {     /* CCFC:35-46 */
    if (r->threshold_type == 1) return r->count;
    const int cc = (r->namespace_idx >= 0 && r->namespace_idx < e->n_ns) ? e->ns[r->namespace_idx].connected_count : 0;
    return r->count * (double)cc;
}

static void tok_free(orc_tok *t) {
    kv_free(&t->index);
    free(t->fid); free(t->acq); free(t->alive);
    memset(t, 0, sizeof(*t));
}

/* One event of ConcurrentClusterFlowChecker (CCFC:48-101) against token cache `tk`; nowCalls lives in
 * the engine's map (values updated in place: the map's layout does not change during a replay). */
static void conc_event(orc_engine *e, orc_tok *tk, const orc_concurrent_event *x, int64_t new_id, int8_t *status,
                       int64_t *token_out) {
    *token_out = 0;
    if (x->kind == 0) {
        if (!(x->flags & 1u) || x->flow_idx == -2 || x->acquire <= 0) { *status = ORC_BAD_REQUEST; return; }
        if (x->flow_idx < 0 || x->flow_idx >= e->n_rules || !e->cm[x->flow_idx]) { *status = ORC_NO_RULE_EXISTS; return; }
        const orc_flow_rule *r = &e->rules[x->flow_idx];
        int64_t *now = kv_find(&e->now_calls, (uint64_t)r->flow_id);
        if (!now) { *status = ORC_FAIL; return; }                                  /* CCFC:51-54 */
        const int32_t sum = (int32_t)((uint32_t)(int32_t)*now + (uint32_t)x->acquire);
        if ((double)sum > conc_threshold(e, r)) { *status = ORC_BLOCKED; return; }  /* CCFC:57-69 */
        *now = (int32_t)((uint32_t)(int32_t)*now + (uint32_t)x->acquire);         /* CCFC:70 */
        if (tk->n == tk->cap) {
            tk->cap = tk->cap ? 2 * tk->cap : 1024;
            tk->fid = (int64_t *)realloc(tk->fid, (size_t)tk->cap * sizeof(int64_t));
            tk->acq = (int32_t *)realloc(tk->acq, (size_t)tk->cap * sizeof(int32_t));
            tk->alive = (uint8_t *)realloc(tk->alive, (size_t)tk->cap);
        }
        tk->fid[tk->n] = r->flow_id;
        tk->acq[tk->n] = x->acquire;
        tk->alive[tk->n] = 1;
        *kv_insert(&tk->index, (uint64_t)new_id, 0) = tk->n++;
        tk->live++;
        *status = ORC_OK;
        *token_out = new_id;
    } else if (x->kind == 1) {
        const int64_t *rec = kv_find(&tk->index, (uint64_t)x->token_id);           /* CCFC:82-86 */
        if (!rec || !tk->alive[*rec]) { *status = 7; return; }                     /* ALREADY_RELEASE */
        if (!kv_find(&e->rule_by_fid, (uint64_t)tk->fid[*rec])) { *status = ORC_NO_RULE_EXISTS; return; }
        tk->alive[*rec] = 0;                                                        /* CCFC:92-98 */
        tk->live--;
        int64_t *now = kv_find(&e->now_calls, (uint64_t)tk->fid[*rec]);
        *now = (int32_t)((uint32_t)(int32_t)*now - (uint32_t)tk->acq[*rec]);
        *status = 6;                                                                /* RELEASE_OK */
    } else {
        *status = ORC_BAD_REQUEST;
    }
}

void orc_concurrent_replay(orc_engine *e, int64_t n, const orc_concurrent_event *ev, const int64_t *new_ids,
                           int8_t *status, int64_t *token_out) {
    for (int64_t i = 0; i < n; i++) conc_event(e, &e->tok, &ev[i], new_ids[i], &status[i], &token_out[i]);
}

/* Flow-sharded multi-threaded concurrency replay (CPU baseline only, SURVEY section 8(d): T threads
 * sharded by flow).  Thread k owns the flows with flow_idx mod T == k and a token cache of its own; a
 * release goes to the thread whose flow issued its token (token -> owner from the acquires that pass
 * with new_ids[i] != 0: a sharded server routes a token id to its shard), an unknown token to thread 0
 * (ALREADY_RELEASE).  Each flow still sees its events in arrival order.  Valid on a fresh engine (no
 * tokens cached before the call); the engine's own token cache is left untouched. */
typedef struct {
    orc_engine *e;
    int64_t n;
    const orc_concurrent_event *ev;
    const int64_t *new_ids;
    const uint8_t *owner;
    int8_t *status;
    int64_t *token_out;
    int k;
} conc_mt_arg;

static void *conc_mt_worker(void *p) {
    conc_mt_arg *a = (conc_mt_arg *)p;
    orc_tok tk;
    memset(&tk, 0, sizeof(tk));
    kv_init(&tk.index);
    for (int64_t i = 0; i < a->n; i++)
        if (a->owner[i] == a->k) conc_event(a->e, &tk, &a->ev[i], a->new_ids[i], &a->status[i], &a->token_out[i]);
    tok_free(&tk);
    return NULL;
}

int orc_concurrent_replay_mt(orc_engine *e, int64_t n, const orc_concurrent_event *ev, const int64_t *new_ids,
                             int8_t *status, int64_t *token_out, int nthreads) {
    if (nthreads > 255) nthreads = 255;
    if (nthreads <= 1) {
        orc_concurrent_replay(e, n, ev, new_ids, status, token_out);
        return 1;
    }
    uint8_t *owner = (uint8_t *)malloc((size_t)(n > 0 ? n : 1));
    kvmap tok_owner;                                       /* token id -> owning thread */
    kv_init(&tok_owner);
    for (int64_t i = 0; i < n; i++) {
        const orc_concurrent_event *x = &ev[i];
        if (x->kind == 0) {
            const int k = x->flow_idx >= 0 ? (int)(x->flow_idx % nthreads) : 0;
            owner[i] = (uint8_t)k;
            if (new_ids[i]) *kv_insert(&tok_owner, (uint64_t)new_ids[i], 0) = k;
        } else {
            const int64_t *k = x->kind == 1 ? kv_find(&tok_owner, (uint64_t)x->token_id) : NULL;
            owner[i] = (uint8_t)(k ? *k : 0);
        }
    }
    pthread_t th[255];
    conc_mt_arg args[255];
    for (int k = 0; k < nthreads; k++) {
        args[k] = (conc_mt_arg){e, n, ev, new_ids, owner, status, token_out, k};
        pthread_create(&th[k], NULL, conc_mt_worker, &args[k]);
    }
    for (int k = 0; k < nthreads; k++) pthread_join(th[k], NULL);
    kv_free(&tok_owner);
    free(owner);
    return nthreads;
}

int32_t orc_concurrent_now_calls(orc_engine *e, int32_t flow_idx) {
    if (flow_idx < 0 || flow_idx >= e->n_rules) return 0;
    const int64_t *now = kv_find(&e->now_calls, (uint64_t)e->rules[flow_idx].flow_id);
    return now ? (int32_t)*now : 0;
}

int64_t orc_concurrent_token_count(orc_engine *e) { return e->tok.live; }

/* RegularExpireStrategy.clearToken with <= executeCount cached tokens: every token qualifies and
 * leaves the cache; nowCalls of a still-present flowId gets the count back (RES:94-136). */
int64_t orc_concurrent_expire_all(orc_engine *e) {
    int64_t removed = 0;
    for (int64_t t = 0; t < e->tok.n; t++) {
        if (!e->tok.alive[t]) continue;
        e->tok.alive[t] = 0;
        e->tok.live--;
        removed++;
        int64_t *now = kv_find(&e->now_calls, (uint64_t)e->tok.fid[t]);
        if (now) *now = (int32_t)((uint32_t)(int32_t)*now - (uint32_t)e->tok.acq[t]);
    }
    return removed;
}
