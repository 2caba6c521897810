/*
 * sentinel_oracle.h -- CPU restatement of Sentinel's sliding-window token-decision path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity checker (and the "port" CPU baseline in
 * bench.py).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it.  The product path (sentinel_amd/, libsentinel_amd.so) never links or calls it.
 *
 * Restated from the reference Java (paths relative to /root/reference), with an injected
 * clock: every call takes the event timestamp `t` that TimeUtil.currentTimeMillis() would
 * have returned (sentinel-core/.../util/TimeUtil.java:49-51).
 *
 * Pinned by the reference's own known-answer tests, transcribed under tests/golden/kat_*.json
 * (see tests/test_oracle_kat.py and DESIGN.md "Oracle").
 */
#ifndef SENTINEL_ORACLE_H
#define SENTINEL_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ClusterFlowEvent ordinals (srv/flow/statistic/data/ClusterFlowEvent.java:22-52). */
enum {
    ORC_PASS = 0, ORC_BLOCK = 1, ORC_PASS_REQUEST = 2, ORC_BLOCK_REQUEST = 3,
    ORC_OCCUPIED_PASS = 4, ORC_OCCUPIED_BLOCK = 5, ORC_WAITING = 6, ORC_NEVENTS = 7
};

/* MetricEvent ordinals (core/slots/statistic/MetricEvent.java:21-39). */
enum {
    ORC_M_PASS = 0, ORC_M_BLOCK = 1, ORC_M_EXCEPTION = 2, ORC_M_SUCCESS = 3,
    ORC_M_RT = 4, ORC_M_OCCUPIED_PASS = 5, ORC_M_NEVENTS = 6
};

/* ---------------- ClusterMetric (srv/flow/statistic/metric/ClusterMetric.java) ---------------- */
typedef struct orc_cluster_metric orc_cluster_metric;
orc_cluster_metric *orc_cm_new(int sample_count, int interval_ms);
void    orc_cm_free(orc_cluster_metric *m);
void    orc_cm_add(orc_cluster_metric *m, int64_t t, int event, int64_t count);
int64_t orc_cm_get_current_count(orc_cluster_metric *m, int64_t t, int event);   /* CM:43-45 */
int64_t orc_cm_get_sum(orc_cluster_metric *m, int64_t t, int event);
double  orc_cm_get_avg(orc_cluster_metric *m, int64_t t, int event);
int     orc_cm_try_occupy_next(orc_cluster_metric *m, int64_t t, int event, int acquire, double threshold);
/* out: sample_count * (1 start + 7 counters) then occupy[7] then has_occupied (1). start=-1 => slot absent */
void    orc_cm_dump(const orc_cluster_metric *m, int64_t *out);
/* LA:330-343 list(validTime).size() -- no roll. */
int     orc_cm_list_count(const orc_cluster_metric *m, int64_t t);
/* CMLA:181-190 getFirstCountOfWindow(event) at time t (LA:399-409 getValidHead). */
int64_t orc_cm_first_count(orc_cluster_metric *m, int64_t t, int event);
/* Current-window start for t after the roll (LA:149-248), -1 for t<0. */
int64_t orc_cm_window_start(orc_cluster_metric *m, int64_t t);

/* ---------------- RequestLimiter (srv/flow/statistic/limit/RequestLimiter.java) ---------------- */
typedef struct orc_limiter orc_limiter;
orc_limiter *orc_limiter_new(double qps_allowed);
void    orc_limiter_free(orc_limiter *l);
void    orc_limiter_add(orc_limiter *l, int64_t t, int x);
int64_t orc_limiter_get_sum(orc_limiter *l, int64_t t);
double  orc_limiter_get_qps(orc_limiter *l, int64_t t);
int     orc_limiter_can_pass(orc_limiter *l, int64_t t);
int     orc_limiter_try_pass(orc_limiter *l, int64_t t);

/* ---------------- ClusterParamMetric (srv/flow/statistic/metric/ClusterParamMetric.java) ------- */
typedef struct orc_param_metric orc_param_metric;
orc_param_metric *orc_pm_new(int sample_count, int interval_ms, int max_capacity);
void    orc_pm_free(orc_param_metric *m);
void    orc_pm_add_value(orc_param_metric *m, int64_t t, uint64_t key, int count);
int64_t orc_pm_get_sum(orc_param_metric *m, int64_t t, uint64_t key);
double  orc_pm_get_avg(orc_param_metric *m, int64_t t, uint64_t key);
/* top-k as in getTopValues: returns k' <= k entries (keys, avg). */
int     orc_pm_top_values(orc_param_metric *m, int64_t t, int number, uint64_t *keys, double *avgs);
int     orc_pm_overflowed(const orc_param_metric *m);   /* 1 if any bucket exceeded max_capacity */

/* ---------------- Rule tables & the token service (DefaultTokenService) ---------------- */
/* Mirrors include/sentinel_amd.h's sentinel_flow_rule_t field-for-field. */
typedef struct {
    int64_t flow_id;            /* ClusterFlowConfig.flowId */
    double  count;              /* FlowRule.count */
    int32_t threshold_type;     /* ClusterRuleConstant: 0 AVG_LOCAL, 1 GLOBAL */
    int32_t sample_count;       /* ClusterFlowConfig.sampleCount (default 10) */
    int32_t window_interval_ms; /* ClusterFlowConfig.windowIntervalMs (default 1000) */
    int32_t namespace_idx;      /* index into the namespace table, -1 = no namespace */
    int32_t checker;            /* 0 = ClusterFlowChecker (TokenService), 1 = SimpleClusterFlowChecker (RLS) */
    int32_t reserved;
} orc_flow_rule;

typedef struct {
    int32_t connected_count;    /* ConnectionManager.getConnectedCount(namespace) */
    int32_t has_limiter;        /* GlobalRequestLimiter.initIfAbsent(namespace) was called */
    double  max_allowed_qps;    /* ServerFlowConfig.maxAllowedQps (default 30000) */
} orc_namespace;

typedef struct {
    double exceed_count;        /* ServerFlowConfig.exceedCount (default 1.0) */
    double max_occupy_ratio;    /* ServerFlowConfig.maxOccupyRatio (default 1.0) */
} orc_server_config;

typedef struct orc_engine orc_engine;
orc_engine *orc_engine_new(const orc_server_config *cfg, const orc_namespace *ns, int n_ns);
void orc_engine_free(orc_engine *e);
/* Returns the number of dense flows (valid rules, one per flowId).  Reload semantics in the .c. */
int  orc_engine_load_flow_rules(orc_engine *e, const orc_flow_rule *rules, int n);
void orc_engine_set_connected_count(orc_engine *e, int32_t ns, int32_t connected);
/* Server window change: every metric (flow and param, orphans included) restarts with it. */
int  orc_engine_reset_metrics(orc_engine *e, int sample_count, int interval_ms);
int  orc_engine_flow_window(const orc_engine *e, int32_t flow_idx, int32_t *out2);
int64_t orc_engine_metric_count(const orc_engine *e);

/* Token-result status codes (core/cluster/TokenResultStatus.java:27-69). */
enum {
    ORC_BAD_REQUEST = -4, ORC_TOO_MANY_REQUEST = -2, ORC_FAIL = -1, ORC_OK = 0,
    ORC_BLOCKED = 1, ORC_SHOULD_WAIT = 2, ORC_NO_RULE_EXISTS = 3
};

/* flow_idx: index into the loaded rule table; -1 => unknown rule (NO_RULE_EXISTS),
 * -2 => invalid id (null or <= 0: BAD_REQUEST).  flags bit0 = prioritized. */
void orc_request_token(orc_engine *e, int32_t flow_idx, int32_t acquire, int prioritized, int64_t t,
                       int8_t *status, int32_t *remaining, int32_t *wait_ms);
/* Sequential replay of a batch in arrival (seq) order. flags may be NULL; wait_ms may be NULL. */
void orc_flow_replay(orc_engine *e, int64_t n, const int32_t *flow_idx, const int32_t *acquire,
                     const uint8_t *flags, const int64_t *ts,
                     int8_t *status, int32_t *remaining, int32_t *wait_ms);
/* Flow-sharded multi-threaded replay (CPU baseline); returns the threads used (1 with limiters). */
int  orc_flow_replay_mt(orc_engine *e, int64_t n, const int32_t *flow_idx, const int32_t *acquire,
                        const uint8_t *flags, const int64_t *ts, int8_t *status, int32_t *remaining,
                        int32_t *wait_ms, int nthreads);
/* Dump flow metric state, orc_cm_dump format. Returns words written or -1. */
int  orc_engine_dump_flow(const orc_engine *e, int32_t flow_idx, int64_t *out);
int64_t orc_engine_limiter_sum(orc_engine *e, int32_t ns, int64_t t);

/* ---- cluster hot-parameter path (ClusterParamFlowChecker) ---- */
typedef struct {
    int64_t flow_id;
    double  count;              /* ParamFlowRule.count */
    int32_t threshold_type;
    int32_t sample_count;
    int32_t window_interval_ms;
    int32_t namespace_idx;
    int32_t hot_begin;          /* [hot_begin, hot_begin+hot_n) into the hot-item arrays */
    int32_t hot_n;
} orc_param_rule;

int  orc_engine_load_param_rules(orc_engine *e, const orc_param_rule *rules, int n,
                                 const uint64_t *hot_keys, const int32_t *hot_counts, int n_hot);
/* One requestParamToken call: values[0..n_values). */
void orc_request_param_token(orc_engine *e, int32_t rule_idx, int32_t acquire, int64_t t,
                             const uint64_t *values, int n_values, int8_t *status, int32_t *remaining);
/* Batch of single-value requests in seq order. */
void orc_param_replay(orc_engine *e, int64_t n, const int32_t *rule_idx, const int32_t *acquire,
                      const uint64_t *param_key, const int64_t *ts, int8_t *status, int32_t *remaining);
/* rule-sharded over nthreads (CPU baseline); returns the threads used */
int  orc_param_replay_mt(orc_engine *e, int64_t n, const int32_t *rule_idx, const int32_t *acquire,
                         const uint64_t *param_key, const int64_t *ts, int8_t *status, int32_t *remaining, int nthreads);
int64_t orc_engine_param_sum(orc_engine *e, int32_t rule_idx, int64_t t, uint64_t key);
int  orc_engine_param_top_values(orc_engine *e, int32_t rule_idx, int64_t t, int number, uint64_t *keys, double *avgs);
int  orc_engine_param_window(const orc_engine *e, int32_t rule_idx, int32_t *out2);
int  orc_engine_param_overflowed(const orc_engine *e);

/* ---------------- Local path: StatisticNode + DefaultController (config 1) ---------------- */
typedef struct orc_stat_node orc_stat_node;
orc_stat_node *orc_node_new(int sample_count, int interval_ms);
void   orc_node_free(orc_stat_node *nd);
double orc_node_pass_qps(orc_stat_node *nd, int64_t t);
int64_t orc_node_pass_sum(orc_stat_node *nd, int64_t t);       /* rollingCounterInSecond.pass() */
int64_t orc_node_block_sum(orc_stat_node *nd, int64_t t);
int64_t orc_node_total_pass(orc_stat_node *nd, int64_t t);     /* rollingCounterInMinute.pass() */
int64_t orc_node_minute_block(orc_stat_node *nd, int64_t t);   /* rollingCounterInMinute.block() */
void   orc_node_add_pass_request(orc_stat_node *nd, int64_t t, int count);
void   orc_node_increase_block_qps(orc_stat_node *nd, int64_t t, int count);
/* DefaultController.canPass(node, acquire) for QPS grade (grade=1) or THREAD grade (0). */
int    orc_default_controller_can_pass(orc_stat_node *nd, double count, int grade, int acquire,
                                       int32_t cur_thread_num, int64_t t);
/* FlowQpsDemo-style replay: for each entry check DefaultController(QPS) then book pass/block
 * like StatisticSlot (core/slots/statistic/StatisticSlot.java:55-116). out_pass[i] = 1/0. */
/* DC:49-76 with a mocked Node value (DefaultControllerTest): cur = passQps or curThreadNum. */
int    orc_default_controller_check(double node_value, double count, int grade, int acquire);
void   orc_local_replay(orc_stat_node *nd, double count, int64_t n, const int32_t *acquire,
                        const int64_t *ts, uint8_t *out_pass);
/* Prioritized entries too (DefaultController.java:52-64 + StatisticNode.tryOccupyNext): out_wait =
 * waitInMs of an occupied pass (0 otherwise). */
void   orc_local_replay_prio(orc_stat_node *nd, double count, int64_t n, const int32_t *acquire,
                             const int64_t *ts, const uint8_t *prio, uint8_t *out_pass, int64_t *out_wait);
int    orc_local_entry(orc_stat_node *nd, double count, int acquire, int prioritized, int64_t t, int64_t *wait);
void   orc_node_set_occupy_timeout(orc_stat_node *nd, int ms);
void   orc_node_set_max_rt(orc_stat_node *nd, int64_t ms);
/* QPS and / or THREAD grade rules (flags), exits, the full metric view: see the .c */
enum { ORC_LR_QPS = 1, ORC_LR_THREAD = 2, ORC_LR_THREAD_FIRST = 4 };
int    orc_local_entry_ex(orc_stat_node *nd, double qps_count, double thread_count, int flags, int acquire,
                          int prioritized, int64_t t, int64_t *wait);
void   orc_local_exit(orc_stat_node *nd, int count, int64_t rt, int error, int64_t t);
void   orc_node_metrics(const orc_stat_node *nd, int64_t t, int64_t *out14);
int64_t orc_node_waiting(orc_stat_node *nd, int64_t t);                 /* rollingCounterInSecond.waiting() */
int64_t orc_node_minute_occupied(orc_stat_node *nd, int64_t t);         /* rollingCounterInMinute.occupiedPass() */
int64_t orc_node_try_occupy_next(orc_stat_node *nd, int64_t t, int acquire, double threshold);
void   orc_node_add_waiting(orc_stat_node *nd, int64_t future_time, int count);
void   orc_node_add_occupied_pass(orc_stat_node *nd, int64_t t, int count);
int64_t orc_node_sec_window_pass(orc_stat_node *nd, int64_t t);
void   orc_node_sec_window_add_pass(orc_stat_node *nd, int64_t t, int n);
int64_t orc_node_sec_values(orc_stat_node *nd, int64_t t, int64_t *sum);

/* ---------------- Local param token bucket (ParamFlowChecker.passDefaultLocalCheck) ----------- */
typedef struct orc_param_bucket orc_param_bucket;
orc_param_bucket *orc_pbucket_new(void);
void orc_pbucket_free(orc_param_bucket *b);
/* token_count = hot-item count or (long)rule.count; returns 1 pass / 0 block. */
int  orc_pbucket_pass_default(orc_param_bucket *b, uint64_t key, int64_t token_count, int64_t burst,
                              int64_t duration_sec, int acquire, int64_t t);

/* ---------------- multi-value cluster params, count-min audit, local param engine ---------------- */
void orc_param_multi_replay(orc_engine *e, int64_t n, const int32_t *rule_idx, const int32_t *acquire,
                            const int64_t *ts, const int32_t *vbegin, const int32_t *vcount,
                            const uint64_t *values, int64_t n_values, int8_t *status, int32_t *remaining);
void orc_param_cm_audit(orc_engine *e, int64_t n, const int32_t *rule_idx, const int32_t *acquire,
                        const int64_t *ts, const int32_t *vbegin, const int32_t *vcount, const uint64_t *values,
                        const int8_t *status_cm, int64_t *violations, int64_t *false_blocks, int64_t *decided);

/* Mirrors include/sentinel_amd.h's sentinel_local_param_rule_t. */
typedef struct {
    double  count;
    int64_t burst_count;
    int64_t duration_in_sec;
    int32_t hot_begin;
    int32_t hot_n;
} orc_local_param_rule;

typedef struct orc_local_engine orc_local_engine;
orc_local_engine *orc_lparam_new(const orc_local_param_rule *rules, int n, const uint64_t *hot_keys,
                                const int32_t *hot_counts, int n_hot);
void orc_lparam_free(orc_local_engine *e);
void orc_lparam_replay(orc_local_engine *e, int64_t n, const int32_t *rule_idx, const int32_t *acquire,
                      const int64_t *ts, const int32_t *vbegin, const int32_t *vcount, const uint64_t *values,
                      int64_t n_values, int8_t *status);
int  orc_lparam_state(orc_local_engine *e, int32_t idx, uint64_t key, int64_t *last, int64_t *tokens);
/* THREAD grade rules (grade 0; default 1 = QPS) and exits (kinds[i] == 1: Entry.exit of a passed
 * entry -> the values' thread counts drop); thread count of a value, -1 when absent. */
void orc_lparam_set_grades(orc_local_engine *e, const int32_t *grade, int n);
void orc_lparam_replay_ex(orc_local_engine *e, int64_t n, const int32_t *rule_idx, const int32_t *acquire,
                          const int64_t *ts, const int32_t *vbegin, const int32_t *vcount, const uint64_t *values,
                          int64_t n_values, const uint8_t *kinds, int8_t *status);
int  orc_lparam_thread_count(orc_local_engine *e, int32_t idx, uint64_t key);

/* ---------------- local rule graph: FlowRuleChecker limitApp / strategy node selection ---------------- */
/* Mirrors include/sentinel_amd.h's sentinel_local_rule_t / sentinel_local_ctx_t. */
enum { ORC_LIMIT_APP_DEFAULT = 0, ORC_LIMIT_APP_OTHER = 1 };
enum { ORC_STRATEGY_DIRECT = 0, ORC_STRATEGY_RELATE = 1, ORC_STRATEGY_CHAIN = 2 };
typedef struct {
    int32_t resource;
    int32_t grade;        /* 1 QPS, 0 THREAD */
    double  count;
    int32_t strategy;     /* 0 DIRECT, 1 RELATE, 2 CHAIN */
    int32_t limit_app;    /* 0 "default", 1 "other", >= 2 an origin id; < 0 blank (-> default) */
    int32_t ref;          /* RELATE: resource index, CHAIN: context id; -1 blank refResource */
    int32_t reserved;
} orc_local_rule;
typedef struct {
    int32_t origin;       /* -1 "" (no origin), 0 "default", 1 "other", >= 2 other names */
    int32_t origin_node;  /* index of ClusterNode(resource).originCountMap[origin] */
    int32_t context;      /* context-name id */
    int32_t default_node; /* index of the DefaultNode of (context, resource) */
} orc_local_ctx;
typedef struct orc_lgraph orc_lgraph;
orc_lgraph *orc_lgraph_new(const orc_local_rule *rules, int n, int n_res, int n_origin_nodes, int n_default_nodes,
                           int sample_count, int interval_ms);
void orc_lgraph_free(orc_lgraph *g);
void orc_lgraph_set_occupy_timeout(orc_lgraph *g, int ms);
int  orc_lgraph_n_rules(const orc_lgraph *g, int res);
int  orc_lgraph_entry(orc_lgraph *g, int res, int acquire, int prioritized, int64_t t, const orc_local_ctx *c,
                      int64_t *wait);
void orc_lgraph_exit(orc_lgraph *g, int res, int count, int64_t rt, int error, int64_t t, const orc_local_ctx *c);
void orc_lgraph_replay(orc_lgraph *g, int64_t n, const int32_t *res, const int32_t *acquire, const int64_t *ts,
                       const orc_local_ctx *ctx, const uint8_t *flags, const int64_t *rt, int8_t *status,
                       int32_t *wait);
int  orc_lgraph_node_metrics(orc_lgraph *g, int kind, int idx, int64_t t, int64_t *out14);

/* ---------------- concurrency tokens (ConcurrentClusterFlowChecker) ---------------- */
/* Mirrors include/sentinel_amd.h's sentinel_concurrent_event_t (kind 0 acquire, 1 release). */
typedef struct {
    int32_t flow_idx;
    int32_t acquire;
    int64_t token_id;
    int32_t kind;
    uint32_t flags;        /* bit0: clientAddress non-empty */
} orc_concurrent_event;

void orc_concurrent_replay(orc_engine *e, int64_t n, const orc_concurrent_event *ev, const int64_t *new_ids,
                           int8_t *status, int64_t *token_out);
/* flow-sharded over nthreads (CPU baseline); returns the threads used */
int  orc_concurrent_replay_mt(orc_engine *e, int64_t n, const orc_concurrent_event *ev, const int64_t *new_ids,
                              int8_t *status, int64_t *token_out, int nthreads);
int32_t orc_concurrent_now_calls(orc_engine *e, int32_t flow_idx);
int64_t orc_concurrent_token_count(orc_engine *e);
int64_t orc_concurrent_expire_all(orc_engine *e);

/* ---------------- Java numerics ---------------- */
int32_t orc_java_d2i(double d);
int64_t orc_java_d2l(double d);
int32_t orc_java_string_hash(const uint16_t *utf16, int64_t n);   /* String.hashCode */

#ifdef __cplusplus
}
#endif
#endif
