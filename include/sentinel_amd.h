/*
 * sentinel_amd.h -- C ABI of the MI355X batched token-decision engine (libsentinel_amd.so).
 *
 * This is the drop-in boundary for Sentinel's cluster token server.  Every entry point below
 * replaces one reference interface (paths relative to the reference repo root):
 *
 *   TokenService.requestToken        sentinel-core/src/main/java/com/alibaba/csp/sentinel/cluster/TokenService.java:36
 *   TokenService.requestParamToken   sentinel-core/src/main/java/com/alibaba/csp/sentinel/cluster/TokenService.java:46
 *   DefaultTokenService              sentinel-cluster/sentinel-cluster-server-default/src/main/java/com/alibaba/csp/sentinel/cluster/flow/DefaultTokenService.java:37-62
 *   ClusterFlowRuleManager (load)    .../cluster/flow/rule/ClusterFlowRuleManager.java:325-372
 *   ClusterParamFlowRuleManager      .../cluster/flow/rule/ClusterParamFlowRuleManager.java:318-360
 *   ClusterServerConfigManager       .../cluster/server/config/ClusterServerConfigManager.java:218-258 (namespace set, limiter)
 *   ServerFlowConfig                 .../cluster/server/config/ServerFlowConfig.java:26-40
 *   ConnectionManager.getConnectedCount .../cluster/server/connection/ConnectionManager.java:47-51
 *   ClusterMetricNodeGenerator       .../cluster/flow/statistic/ClusterMetricNodeGenerator.java:70-86 (snapshot)
 *   SimpleClusterFlowChecker (RLS)   sentinel-cluster/sentinel-cluster-server-envoy-rls/.../rls/flow/SimpleClusterFlowChecker.java:33-65
 *
 * Conventions: plain C types only; every call returns 0 on success or a negative
 * SENTINEL_E_* code (message via sentinel_last_error()).  An engine that cannot run (no GPU,
 * device fault) answers every event with status FAIL (-1) and returns SENTINEL_E_DEVICE, so the
 * reference clients' fallbackToLocalWhenFail path (FlowRuleChecker.java:166-209) still works.
 * Time is explicit: every event carries the millisecond timestamp the reference would have read
 * from TimeUtil.currentTimeMillis() (sentinel-core/.../util/TimeUtil.java:49-51).
 */
#ifndef SENTINEL_AMD_H
#define SENTINEL_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* TokenResultStatus (sentinel-core/.../cluster/TokenResultStatus.java:27-69) */
#define SENTINEL_STATUS_BAD_REQUEST       (-4)
#define SENTINEL_STATUS_TOO_MANY_REQUEST  (-2)
#define SENTINEL_STATUS_FAIL              (-1)
#define SENTINEL_STATUS_OK                (0)
#define SENTINEL_STATUS_BLOCKED           (1)
#define SENTINEL_STATUS_SHOULD_WAIT       (2)
#define SENTINEL_STATUS_NO_RULE_EXISTS    (3)

/* Special flow/rule indices in an event (the host maps flowId -> dense index). */
#define SENTINEL_IDX_NO_RULE   (-1)   /* flowId not loaded   -> NO_RULE_EXISTS */
#define SENTINEL_IDX_BAD_ID    (-2)   /* flowId null or <= 0 -> BAD_REQUEST    */

/* ClusterRuleConstant (sentinel-core/.../slots/block/ClusterRuleConstant.java:27-28) */
#define SENTINEL_THRESHOLD_AVG_LOCAL  0
#define SENTINEL_THRESHOLD_GLOBAL     1

/* Which reference checker decides a flow. */
#define SENTINEL_CHECKER_CLUSTER  0   /* ClusterFlowChecker via DefaultTokenService */
#define SENTINEL_CHECKER_SIMPLE   1   /* SimpleClusterFlowChecker (Envoy RLS)       */

/* Event flags */
#define SENTINEL_FLAG_PRIORITIZED  1u /* requestToken(..., prioritized=true) */

/* Error codes */
#define SENTINEL_OK            0
#define SENTINEL_E_INVALID    (-1)
#define SENTINEL_E_DEVICE     (-2)
#define SENTINEL_E_NOMEM      (-3)
#define SENTINEL_E_STATE      (-4)

/* Number of ClusterFlowEvent counters per bucket (ClusterFlowEvent.java:22-52):
 * PASS, BLOCK, PASS_REQUEST, BLOCK_REQUEST, OCCUPIED_PASS, OCCUPIED_BLOCK, WAITING */
#define SENTINEL_NEVENTS 7

typedef struct sentinel_engine sentinel_engine_t;

/* ServerFlowConfig (ServerFlowConfig.java:26-40). Defaults: 1.0, 1.0. */
typedef struct {
    double exceed_count;
    double max_occupy_ratio;
} sentinel_server_config_t;

/* One namespace of the server namespace set. */
typedef struct {
    int32_t connected_count;   /* ConnectionManager.getConnectedCount(namespace) */
    int32_t has_limiter;       /* GlobalRequestLimiter.initIfAbsent(namespace) was called */
    double  max_allowed_qps;   /* RequestLimiter qpsAllowed (ServerFlowConfig.maxAllowedQps, default 30000) */
} sentinel_namespace_t;

/* A cluster FlowRule as loaded by ClusterFlowRuleManager.applyClusterFlowRule. */
typedef struct {
    int64_t flow_id;             /* ClusterFlowConfig.flowId (> 0) */
    double  count;               /* FlowRule.count (>= 0) */
    int32_t threshold_type;      /* SENTINEL_THRESHOLD_* (ClusterFlowConfig.thresholdType) */
    int32_t sample_count;        /* ClusterFlowConfig.sampleCount (default 10) */
    int32_t window_interval_ms;  /* ClusterFlowConfig.windowIntervalMs (default 1000) */
    int32_t namespace_idx;       /* index into the namespace table; -1 = no namespace */
    int32_t checker;             /* SENTINEL_CHECKER_* */
    int32_t reserved;
} sentinel_flow_rule_t;

/* A cluster ParamFlowRule (ClusterParamFlowRuleManager.java:318-360).  Hot items are passed as
 * parallel arrays; [hot_begin, hot_begin + hot_n) indexes them. */
typedef struct {
    int64_t flow_id;
    double  count;               /* ParamFlowRule.count */
    int32_t threshold_type;
    int32_t sample_count;
    int32_t window_interval_ms;
    int32_t namespace_idx;
    int32_t hot_begin;
    int32_t hot_n;
} sentinel_param_rule_t;

/* TokenResult (sentinel-core/.../cluster/TokenResult.java:26-98), the per-call result. */
typedef struct {
    int32_t status;
    int32_t remaining;
    int32_t wait_in_ms;
    int32_t reserved;
} sentinel_token_result_t;

/* ClusterMetricNode subset produced by the snapshot (ClusterMetricNodeGenerator.java:70-86). */
typedef struct {
    int64_t flow_id;
    double  pass_qps;
    double  block_qps;
} sentinel_flow_snapshot_t;

/* ---- lifecycle ---- */
int  sentinel_engine_create(int device, const sentinel_server_config_t *cfg, sentinel_engine_t **out);
int  sentinel_engine_destroy(sentinel_engine_t *eng);
const char *sentinel_last_error(void);
int  sentinel_device_count(void);

/* ---- rules & config (host-side tables, uploaded to HBM) ---- */
int  sentinel_set_server_config(sentinel_engine_t *eng, const sentinel_server_config_t *cfg);
int  sentinel_set_namespaces(sentinel_engine_t *eng, const sentinel_namespace_t *ns, int32_t n);
int  sentinel_set_connected_count(sentinel_engine_t *eng, int32_t namespace_idx, int32_t connected);
/* Loads the flow rule table: ClusterFlowRuleManager.applyClusterFlowRule (ClusterFlowRuleManager.java:
 * 325-372) over every namespace at once.  Invalid rules (FlowRuleUtil.isValidRule: flowId <= 0,
 * count < 0, bad window config) are dropped; a repeated flowId keeps its first position and its
 * last rule.  ClusterMetricStatistics.putMetricIfAbsent: a flowId present before and after keeps
 * its metric -- its OLD window and counters -- and its nowCalls; a new flowId gets the window of
 * its first occurrence; a flowId that left loses its metric, unless its namespace's list (raw
 * rules of that namespace_idx, valid or not) is empty: then the metric is kept aside (clearAndResetRulesFor
 * leaves METRIC_MAP alone) and comes back if the flowId is loaded again.  The window state moves on
 * the device; the previous table stays in place if anything fails.  Param rules: the same. */
int  sentinel_load_flow_rules(sentinel_engine_t *eng, const sentinel_flow_rule_t *rules, int32_t n);
int  sentinel_load_param_rules(sentinel_engine_t *eng, const sentinel_param_rule_t *rules, int32_t n,
                               const uint64_t *hot_keys, const int32_t *hot_counts, int32_t n_hot);
int32_t sentinel_flow_count(sentinel_engine_t *eng);
int32_t sentinel_param_count(sentinel_engine_t *eng);   /* dense param rules (valid, one per flowId) */
/* flowId -> dense index (or SENTINEL_IDX_NO_RULE / SENTINEL_IDX_BAD_ID), host side. */
int  sentinel_lookup_flow_idx(sentinel_engine_t *eng, int64_t n, const int64_t *flow_ids, int32_t *idx_out);
int  sentinel_lookup_param_idx(sentinel_engine_t *eng, int64_t n, const int64_t *flow_ids, int32_t *idx_out);

/* ---- the batched hot path: DefaultTokenService.requestToken over a batch ----
 * Events in arrival (seq) order; verdicts land at the same positions.  Verdicts equal a
 * sequential replay of the batch through the reference checker with the given timestamps. */

/* One requestToken call (TokenService.java:36): ruleId -> dense flow index (see lookup), acquireCount,
 * and the TimeUtil.currentTimeMillis() value of the call.  16 bytes. */
typedef struct {
    int32_t flow_idx;
    int32_t acquire;
    int64_t ts;
} sentinel_event_t;

/* One single-value requestParamToken call (TokenService.java:46).  param_key is the host's
 * injective 64-bit encoding of (rule, Java-typed value); 0xFFFFFFFFFFFFFFFF is reserved.  24 bytes. */
typedef struct {
    int32_t rule_idx;
    int32_t acquire;
    int64_t ts;
    uint64_t param_key;
} sentinel_param_event_t;

/* Packed TokenResult {status, remaining, waitInMs}: one 8-byte store per event. */
typedef struct {
    int32_t  remaining;
    int16_t  status;
    uint16_t wait_in_ms;
} sentinel_verdict_t;

/* DEVICE pointers; flags (bit0 = prioritized) may be NULL; `stream` is a hipStream_t (NULL = the
 * engine's stream).  Asynchronous. */
/* Several device-resident batches decided in order on `stream` under one engine lock (one call for a
 * batcher's queue of device batches); verdicts and counters equal submitting them one by one. */
int  sentinel_submit_flow_batches(sentinel_engine_t *eng, int32_t n_batches, const int64_t *n,
                                  const sentinel_event_t *const *events, const uint8_t *const *flags,
                                  sentinel_verdict_t *const *verdicts, void *stream);
int  sentinel_submit_flow_batch(sentinel_engine_t *eng, int64_t n, const sentinel_event_t *events,
                                const uint8_t *flags, sentinel_verdict_t *verdicts, void *stream);
/* Same with HOST pointers (pinned or pageable): H2D, decide, D2H, synchronous. */
int  sentinel_submit_flow_batch_host(sentinel_engine_t *eng, int64_t n, const sentinel_event_t *events,
                                     const uint8_t *flags, sentinel_verdict_t *verdicts);
/* Decide-order output: the same decisions and window counters as sentinel_submit_flow_batch, but
 * verdicts[j] answers the event at arrival position seq[j] (seq is a permutation of [0, n)) instead of
 * the event at position j.  The reference answers each requestToken call on its own connection, keyed
 * by the request's xid (srv/server/handler/TokenServerHandler.java:61-81, ClusterResponse), so a
 * consumer that routes every verdict by its seq -- the batcher and the wire server do -- never needs
 * arrival order.  The partition path then writes every flow range's verdicts to its own contiguous
 * positions (whole lines) instead of 8-byte stores scattered over the batch; batches it does not take
 * (small, skewed, namespace limiters) come back in arrival order with seq = identity.  DEVICE pointers
 * (verdicts n x 8 B, seq n x 4 B), asynchronous; the _host variant is H2D, decide, D2H, synchronous. */
int  sentinel_submit_flow_batch_ordered(sentinel_engine_t *eng, int64_t n, const sentinel_event_t *events,
                                        const uint8_t *flags, sentinel_verdict_t *verdicts, uint32_t *seq,
                                        void *stream);
int  sentinel_submit_flow_batch_ordered_host(sentinel_engine_t *eng, int64_t n, const sentinel_event_t *events,
                                             const uint8_t *flags, sentinel_verdict_t *verdicts, uint32_t *seq);
/* Host-fed stream (the north star's pinned host ring + hipMemcpyAsync double-buffering on side
 * streams): decides n HOST events as consecutive batches of `batch` events, batch i+1's H2D and
 * batch i-1's D2H overlapping batch i's decide.  Verdicts equal one sequential replay of all n events
 * (= sentinel_submit_flow_batch_host over all n).  `batch_ms` (optional, ceil(n / batch) floats):
 * per-batch latency, H2D start -> verdicts in host memory.  Pass pinned memory for overlap. */
int  sentinel_submit_flow_stream_host(sentinel_engine_t *eng, int64_t n, const sentinel_event_t *events,
                                      const uint8_t *flags, sentinel_verdict_t *verdicts, int64_t batch,
                                      float *batch_ms);
int  sentinel_submit_param_batch(sentinel_engine_t *eng, int64_t n, const sentinel_param_event_t *events,
                                 sentinel_verdict_t *verdicts, void *stream);
int  sentinel_submit_param_batch_host(sentinel_engine_t *eng, int64_t n, const sentinel_param_event_t *events,
                                      sentinel_verdict_t *verdicts);
/* Decide-order output for single-value requestParamToken batches (TokenService.java:46), as
 * sentinel_submit_flow_batch_ordered: verdicts[j] answers the request at arrival position seq[j].  The
 * partition-local key walks (exact slots and the shared count-min sketch) write each (rule, value) key's
 * verdicts at its grouped positions; other paths answer in arrival order with seq = identity.  The wire
 * server's PARAM requests (TokenServerHandler.java:61-81, one response per xid) take it. */
int  sentinel_submit_param_batch_ordered(sentinel_engine_t *eng, int64_t n, const sentinel_param_event_t *events,
                                         sentinel_verdict_t *verdicts, uint32_t *seq, void *stream);
int  sentinel_submit_param_batch_ordered_host(sentinel_engine_t *eng, int64_t n, const sentinel_param_event_t *events,
                                              sentinel_verdict_t *verdicts, uint32_t *seq);

/* ---- hot-parameter requests beyond one value, count-min mode, local token bucket ---- */

/* One requestParamToken call with any number of values (TokenService.java:46;
 * ClusterParamFlowChecker.acquireClusterToken, sentinel-cluster/.../cluster/flow/ClusterParamFlowChecker.java:42-87),
 * or one local ParamFlowChecker.passLocalCheck over a collection / array argument
 * (sentinel-extension/sentinel-parameter-flow-control/.../param/ParamFlowChecker.java:78-103).
 * Its values are values[value_begin, value_begin + value_count) of the batch's value array, each
 * the host's injective 64-bit encoding of (rule, Java-typed value).  24 bytes; the first 16 are
 * laid out like sentinel_event_t. */
typedef struct {
    int32_t rule_idx;
    int32_t acquire;
    int64_t ts;
    int32_t value_begin;
    int32_t value_count;
} sentinel_param_multi_event_t;

/* Cluster param requests with value lists: the values are checked in order, the first whose
 * remaining would be negative blocks the request and no counter is touched; otherwise every
 * value's counter is incremented (a repeated value twice).  remaining is that of the last value,
 * -1 for more than one value (CPFC:81-84).  Events of one rule are decided in arrival order by
 * one lane, so mixing them with single-value batches keeps the sequential semantics.  DEVICE
 * pointers, asynchronous. */
int  sentinel_submit_param_multi_batch(sentinel_engine_t *eng, int64_t n, const sentinel_param_multi_event_t *events,
                                       const uint64_t *values, int64_t n_values, sentinel_verdict_t *verdicts,
                                       void *stream);
int  sentinel_submit_param_multi_batch_host(sentinel_engine_t *eng, int64_t n, const sentinel_param_multi_event_t *events,
                                            const uint64_t *values, int64_t n_values, sentinel_verdict_t *verdicts);

/* Counter mode of the cluster param path (BASELINE config 4).  COUNT_MIN keeps, per rule, a
 * depth x width sketch of window counters instead of exact per-value counters: memory is bounded
 * whatever the number of values, estimates never undercount a value's own passes, so a request may
 * be blocked that exact counters would pass but never the reverse; with probability >= 1 -
 * exp(-depth) an estimate exceeds the true window count by at most (e / width) x (the rule's total
 * window count).  Switching modes clears the param counters. */
#define SENTINEL_PARAM_EXACT      0
#define SENTINEL_PARAM_COUNT_MIN  1
/* One depth x width sketch for every param rule (keys are unique per (rule, value)): memory
 * independent of the rule count; the bound is (e / width) x (the total window count of all rules).
 * Needs one window (sampleCount, intervalMs) for every param rule: a per-rule window could reset a
 * cell slot another rule's window still counts.  Single-value batches are decided one (rule, value)
 * key per lane: a request's estimate is the cells as the earlier batches left them plus its own key's
 * admitted count in this batch (other keys' counts of the same batch are added after it), still never
 * below the exact count; precondition: request timestamps do not go back across batches. */
#define SENTINEL_PARAM_COUNT_MIN_SHARED  2
int  sentinel_set_param_mode(sentinel_engine_t *eng, int32_t mode, int32_t depth, int32_t width);

/* Local hot-parameter rule (ParamFlowRule, QPS grade, default control behaviour) as
 * ParamFlowChecker.passDefaultLocalCheck reads it (ParamFlowChecker.java:127-202).  Rule index =
 * position in the loaded array; rules failing ParamFlowRuleUtil.isValidRule
 * (ParamFlowRuleUtil.java:46-52) answer NO_RULE_EXISTS.  32 bytes. */
typedef struct {
    double  count;             /* ParamFlowRule.count: tokenCount = (long) count */
    int64_t burst_count;       /* ParamFlowRule.burstCount */
    int64_t duration_in_sec;   /* ParamFlowRule.durationInSec */
    int32_t hot_begin;         /* [hot_begin, hot_begin + hot_n) into the hot-item arrays */
    int32_t hot_n;
} sentinel_local_param_rule_t;

/* Loads the local rules; every token bucket restarts (ParameterMetric counters). */
int  sentinel_load_local_param_rules(sentinel_engine_t *eng, const sentinel_local_param_rule_t *rules, int32_t n,
                                     const uint64_t *hot_keys, const int32_t *hot_counts, int32_t n_hot);
/* passLocalCheck per event: OK (pass) or BLOCKED; an empty value list passes. */
int  sentinel_submit_local_param_batch(sentinel_engine_t *eng, int64_t n, const sentinel_param_multi_event_t *events,
                                       const uint64_t *values, int64_t n_values, sentinel_verdict_t *verdicts,
                                       void *stream);
int  sentinel_submit_local_param_batch_host(sentinel_engine_t *eng, int64_t n, const sentinel_param_multi_event_t *events,
                                            const uint64_t *values, int64_t n_values, sentinel_verdict_t *verdicts);
/* Token bucket of one value: {lastAddTokenTime, tokens} (-1 when absent); returns 1 if present.
 * For a THREAD grade rule `tokens` is the value's thread count (-1: no entry in the map). */
int  sentinel_local_param_state(sentinel_engine_t *eng, uint64_t param_key, int64_t *last_add_ms, int64_t *tokens);
/* Grades of the loaded local rules (ParamFlowRule.grade: 1 QPS = the token bucket above, 0 THREAD);
 * reset to all-QPS by every sentinel_load_local_param_rules.  A THREAD rule's check passes iff every
 * value's thread count + 1 <= its threshold (hot-item count, else (long) count:
 * ParamFlowChecker.passSingleValueCheck, ParamFlowChecker.java:112-122); a passing check adds one to
 * every value (the entry callback, ParameterMetric.addThreadCount, ParameterMetric.java:184-239).
 * Counts live per param key, so a rule's keys should encode (resource, paramIdx, value) -- the
 * reference shares one map per param index (exact when one param rule reads an index). */
int  sentinel_set_local_param_grades(sentinel_engine_t *eng, const int32_t *grades, int32_t n);
/* Local param batch with event kinds: kinds[i] == 1 is Entry.exit of a passed entry -- its values'
 * thread counts drop by one, removed at 0 (ParameterMetric.decreaseThreadCount,
 * ParameterMetric.java:125-181; answers OK, no-op for QPS rules); anything else a check as in
 * sentinel_submit_local_param_batch.  kinds may be NULL (all checks). */
int  sentinel_submit_local_param_batch_ex(sentinel_engine_t *eng, int64_t n, const sentinel_param_multi_event_t *events,
                                          const uint8_t *kinds, const uint64_t *values, int64_t n_values,
                                          sentinel_verdict_t *verdicts, void *stream);
int  sentinel_submit_local_param_batch_ex_host(sentinel_engine_t *eng, int64_t n, const sentinel_param_multi_event_t *events,
                                               const uint8_t *kinds, const uint64_t *values, int64_t n_values,
                                               sentinel_verdict_t *verdicts);

/* ---- local SphU.entry admission: DefaultController over a resource's ClusterNode ----
 * FlowSlot -> FlowRuleChecker.passLocalCheck -> DefaultController.canPass (QPS grade, limitApp
 * "default", strategy DIRECT: sentinel-core/.../slots/block/flow/FlowRuleChecker.java:44-132,
 * controller/DefaultController.java:49-76) and StatisticSlot's booking into the StatisticNode's
 * second window (SampleCountProperty x IntervalProperty) and minute window (60 x 1 s)
 * (sentinel-core/.../slots/statistic/StatisticSlot.java:55-116, node/StatisticNode.java:96-264). */
typedef struct {
    double  count;       /* the smallest count of the resource's QPS FlowRules (every rule must pass) */
    int32_t has_rule;    /* 0: no flow rule -> every entry passes (and is counted) */
    int32_t reserved;
} sentinel_local_resource_t;

/* Loads the resources (index = position) with the node window config (defaults 2, 1000); every
 * node starts empty.  Precondition (documented): <= 6000 resources (CtSph MAX_SLOT_CHAIN_SIZE). */
int  sentinel_load_local_resources(sentinel_engine_t *eng, const sentinel_local_resource_t *res, int32_t n,
                                   int32_t sample_count, int32_t interval_ms);
/* Events {resource index, acquireCount, ts} + optional prioritized flags (SphU.entryWithPriority,
 * bit 0): OK (entry) or BLOCKED (FlowException); an unknown resource answers NO_RULE_EXISTS.  A
 * prioritized entry over the limit that StatisticNode.tryOccupyNext can place in a future window
 * (DefaultController.java:52-64) answers OK with waitInMs = the wait (PriorityWaitException: the
 * caller sleeps, then the entry passes).  Replaces SphU.entry(...) -> ... -> FlowSlot ->
 * DefaultController.canPass and StatisticSlot.entry's booking (StatisticSlot.java:55-116). */
int  sentinel_submit_local_entry_batch(sentinel_engine_t *eng, int64_t n, const sentinel_event_t *events,
                                       const uint8_t *prioritized, sentinel_verdict_t *verdicts, void *stream);
int  sentinel_submit_local_entry_batch_host(sentinel_engine_t *eng, int64_t n, const sentinel_event_t *events,
                                            const uint8_t *prioritized, sentinel_verdict_t *verdicts);
/* {second-window PASS, BLOCK, minute-window PASS, BLOCK, minute OCCUPIED_PASS, waiting()} of a
 * resource's node at ts (read-only view, no roll). */
int  sentinel_local_node_stats(sentinel_engine_t *eng, int32_t resource_idx, int64_t ts, int64_t *out6);
/* OccupyTimeoutProperty.updateTimeout (OccupyTimeoutProperty.java:64-78): values < 0 or above the
 * node interval are ignored (default 500 ms). */
int  sentinel_set_occupy_timeout(sentinel_engine_t *eng, int32_t timeout_ms);

/* Resources with QPS and / or THREAD grade DefaultController rules (FlowRuleChecker.checkFlow checks
 * a resource's rules in order; every rule of a grade must pass, so the smallest count of each grade
 * decides).  THREAD: cur = (int) curThreadNum (StatisticNode.java:241-243), block iff
 * (double)(cur + acquire) > count (DefaultController.java:49-51).  The prioritized occupy path only
 * follows a failing QPS rule, and skips the rules after it, hence THREAD_FIRST.  Counts < 0 drop the
 * rule (FlowRuleUtil.isValidRule).  24 bytes. */
#define SENTINEL_LOCAL_QPS           1
#define SENTINEL_LOCAL_THREAD        2
#define SENTINEL_LOCAL_THREAD_FIRST  4
typedef struct {
    double  qps_count;
    double  thread_count;
    int32_t flags;       /* SENTINEL_LOCAL_* */
    int32_t reserved;
} sentinel_local_resource_ex_t;
int  sentinel_load_local_resources_ex(sentinel_engine_t *eng, const sentinel_local_resource_ex_t *res, int32_t n,
                                      int32_t sample_count, int32_t interval_ms);

/* A local batch of entries and exits.  flags[i]: bit 0 prioritized entry, bit 1 EXIT -- Entry.exit
 * of an entry that passed (StatisticSlot.exit, StatisticSlot.java:126-164; a blocked entry's exit
 * books nothing and must not be sent): at ts, SUCCESS += acquire and RT += rt_ms[i] in the second
 * and minute windows (StatisticNode.addRtAndSuccess, StatisticNode.java:252-258; each bucket keeps
 * its minRt, MetricBucket.java:132-139), curThreadNum -= 1, and with bit 2 (a business exception
 * traced on the entry: Tracer.trace -> Entry.setError) EXCEPTION += acquire.  An entry that passes
 * adds one thread (StatisticSlot.java:62, 82).  Exits answer OK.  flags / rt_ms may be NULL (plain
 * entries).  Events of one resource are applied in arrival order. */
int  sentinel_submit_local_batch(sentinel_engine_t *eng, int64_t n, const sentinel_event_t *events, const uint8_t *flags,
                                 const int64_t *rt_ms, sentinel_verdict_t *verdicts, void *stream);
int  sentinel_submit_local_batch_host(sentinel_engine_t *eng, int64_t n, const sentinel_event_t *events,
                                      const uint8_t *flags, const int64_t *rt_ms, sentinel_verdict_t *verdicts);
/* Read-only view of a resource's node at ts as a roll at ts would leave it: out[0..5] second window
 * {PASS, BLOCK, EXCEPTION, SUCCESS, RT, minRt}, out[6..12] minute window {PASS, BLOCK,
 * OCCUPIED_PASS, EXCEPTION, SUCCESS, RT, minRt}, out[13] curThreadNum.  minRt as ArrayMetric.minRt
 * (ArrayMetric.java:142-153): max(1, min(statisticMaxRt, the valid buckets' minRt)). */
int  sentinel_local_node_metrics(sentinel_engine_t *eng, int32_t resource_idx, int64_t ts, int64_t *out14);
/* SentinelConfig.statisticMaxRt (default 5000 ms): a fresh bucket's minRt. */
int  sentinel_set_statistic_max_rt(sentinel_engine_t *eng, int64_t max_rt_ms);

/* ---- local rule graph: FlowRuleChecker with every limitApp and strategy ----
 * Replaces FlowSlot -> FlowRuleChecker.checkFlow / selectNodeByRequesterAndStrategy /
 * selectReferenceNode (sentinel-core/.../slots/block/flow/FlowRuleChecker.java:44-145) over the nodes
 * the slot chain builds: a ClusterNode per resource, created by the resource's first entry
 * (ClusterBuilderSlot.java:74-92); an origin StatisticNode per (resource, origin)
 * (ClusterNode.getOrCreateOriginNode, ClusterNode.java:101-118); a DefaultNode per (context, resource)
 * (NodeSelectorSlot) whose thread / pass / block / RT / exception booking also reaches the ClusterNode
 * (DefaultNode.java:110-143).  Rule selection (limitApp, STRATEGY_DIRECT / RELATE / CHAIN):
 *   limitApp == origin (not "default" / "other"): DIRECT -> origin node, else the reference node
 *   limitApp "default":                            DIRECT -> ClusterNode, else the reference node
 *   limitApp "other", origin matched by no rule of the resource (FlowRuleManager.isOtherOrigin):
 *                                                  DIRECT -> origin node, else the reference node
 *   reference node: RELATE -> the refResource's ClusterNode (none before its first entry),
 *                   CHAIN  -> this DefaultNode iff the context name is refResource;  no node -> pass.
 * The caller interns strings: origin / limitApp ids 0 = "default", 1 = "other", >= 2 any other name,
 * -1 = "" (no origin; as a limitApp: blank -> "default"); context-name ids are the CHAIN refResource
 * ids; node indices are the caller's dense numbering of (resource, origin) and (context, resource). */
#define SENTINEL_LIMIT_APP_DEFAULT  0
#define SENTINEL_LIMIT_APP_OTHER    1
#define SENTINEL_STRATEGY_DIRECT    0
#define SENTINEL_STRATEGY_RELATE    1
#define SENTINEL_STRATEGY_CHAIN     2
#define SENTINEL_GRADE_THREAD       0
#define SENTINEL_GRADE_QPS          1
#define SENTINEL_NODE_CLUSTER       0
#define SENTINEL_NODE_ORIGIN        1
#define SENTINEL_NODE_DEFAULT       2
typedef struct {
    int32_t resource;    /* FlowRule.resource as a resource index */
    int32_t grade;       /* SENTINEL_GRADE_* (FlowRule.grade) */
    double  count;
    int32_t strategy;    /* SENTINEL_STRATEGY_* */
    int32_t limit_app;   /* limitApp id (see above) */
    int32_t ref;         /* RELATE: refResource index, CHAIN: refResource context id, -1 blank */
    int32_t reserved;
} sentinel_local_rule_t;           /* 32 bytes */
typedef struct {
    int32_t origin;        /* context origin id, -1 = "" */
    int32_t origin_node;   /* index of the (resource, origin) node; ignored when origin == -1 */
    int32_t context;       /* context-name id */
    int32_t default_node;  /* index of the (context, resource) DefaultNode */
} sentinel_local_ctx_t;            /* 16 bytes, one per event */
/* Loads FlowRuleManager.loadRules' rules (DefaultController, controlBehavior default): invalid ones
 * dropped as FlowRuleUtil.isValidRule (count < 0, grade not QPS / THREAD, a QPS RELATE / CHAIN rule
 * with a blank refResource; FlowRuleUtil.java:167-238), duplicates dropped (buildFlowRuleMap's
 * HashSet), then FlowRuleComparator's stable sort (non-"default" limitApps first,
 * FlowRuleComparator.java:30-55): pass each resource's rules in FlowRuleManager's order.  Every node
 * (n_res ClusterNodes, n_origin_nodes, n_default_nodes) starts empty and no ClusterNode exists yet.
 * The node windows are SampleCountProperty x IntervalProperty as sentinel_load_local_resources. */
int  sentinel_load_local_rules(sentinel_engine_t *eng, const sentinel_local_rule_t *rules, int32_t n, int32_t n_res,
                               int32_t n_origin_nodes, int32_t n_default_nodes, int32_t sample_count,
                               int32_t interval_ms);
/* A batch of SphU.entry / Entry.exit events with their contexts (flags and rt_ms as
 * sentinel_submit_local_batch): every rule checked in order on its selected node (DefaultController,
 * the prioritized occupy path included), then StatisticSlot's booking on the DefaultNode (+ the
 * ClusterNode) and the origin node (StatisticSlot.java:55-164; the global ENTRY_NODE of EntryType.IN,
 * read only by SystemSlot, is not kept).  A bad resource or node index answers NO_RULE_EXISTS, ts < 0
 * FAIL.  Resources joined by RELATE rules are decided in one arrival-ordered pass. */
int  sentinel_submit_local_graph_batch(sentinel_engine_t *eng, int64_t n, const sentinel_event_t *events,
                                       const sentinel_local_ctx_t *ctx, const uint8_t *flags, const int64_t *rt_ms,
                                       sentinel_verdict_t *verdicts, void *stream);
int  sentinel_submit_local_graph_batch_host(sentinel_engine_t *eng, int64_t n, const sentinel_event_t *events,
                                            const sentinel_local_ctx_t *ctx, const uint8_t *flags,
                                            const int64_t *rt_ms, sentinel_verdict_t *verdicts);
/* sentinel_local_node_metrics of any node: kind SENTINEL_NODE_CLUSTER (resource index),
 * SENTINEL_NODE_ORIGIN, SENTINEL_NODE_DEFAULT. */
int  sentinel_local_graph_node_metrics(sentinel_engine_t *eng, int32_t kind, int32_t idx, int64_t ts, int64_t *out14);

/* ---- cluster concurrency tokens (thread grade): TokenService.requestConcurrentToken /
 *      releaseConcurrentToken (TokenService.java:56,62) -> ConcurrentClusterFlowChecker
 *      (sentinel-cluster/.../cluster/flow/ConcurrentClusterFlowChecker.java:48-101) ---- */
#define SENTINEL_STATUS_RELEASE_OK       6    /* TokenResultStatus.RELEASE_OK */
#define SENTINEL_STATUS_ALREADY_RELEASE  7    /* TokenResultStatus.ALREADY_RELEASE */
#define SENTINEL_CONCURRENT_ACQUIRE  0
#define SENTINEL_CONCURRENT_RELEASE  1
#define SENTINEL_CONCURRENT_HAS_ADDRESS 1u    /* flags: clientAddress non-null and non-empty (DTS:89-91) */

/* One acquire (flow_idx from sentinel_lookup_flow_idx, acquire count, flags) or release (token_id).
 * 24 bytes. */
typedef struct {
    int32_t flow_idx;
    int32_t acquire;
    int64_t token_id;
    int32_t kind;
    uint32_t flags;
} sentinel_concurrent_event_t;

/* TokenResult of a concurrent call: status OK with a fresh token id, BLOCKED, BAD_REQUEST,
 * NO_RULE_EXISTS, FAIL (token cache full), RELEASE_OK or ALREADY_RELEASE.  16 bytes. */
typedef struct {
    int64_t token_id;
    int32_t status;
    int32_t reserved;
} sentinel_concurrent_result_t;

/* A batch of acquires / releases in arrival order; each flow's events are decided in order (HOST
 * pointers, synchronous).  Token ids are engine-generated opaque 64-bit values (the reference draws
 * them from UUID.randomUUID(), TokenCacheNode.java:63). */
int  sentinel_submit_concurrent_batch_host(sentinel_engine_t *eng, int64_t n, const sentinel_concurrent_event_t *events,
                                           sentinel_concurrent_result_t *results);
/* The same on DEVICE pointers, asynchronous on `stream` (null: the engine's stream), like
 * sentinel_submit_flow_batch: replaces a batch of TokenService.requestConcurrentToken /
 * releaseConcurrentToken calls (TokenService.java:56,62; DefaultTokenService.java:64-83).  A release
 * names a token issued by an earlier batch (token ids come back with the results); the first release
 * of a token in a batch finds it, later ones answer ALREADY_RELEASE.  The token cache is kept below 3/4
 * full from a host-side bound; a batch that could cross it synchronises and compacts the cache. */
int  sentinel_submit_concurrent_batch(sentinel_engine_t *eng, int64_t n, const sentinel_concurrent_event_t *events,
                                      sentinel_concurrent_result_t *results, void *stream);
/* CurrentConcurrencyManager.get(flowId) of a loaded flow. */
int  sentinel_concurrent_now_calls(sentinel_engine_t *eng, int32_t flow_idx, int32_t *now_calls);
/* TokenCacheNodeManager.getSize(). */
int  sentinel_concurrent_token_count(sentinel_engine_t *eng, int64_t *count);
/* One RegularExpireStrategy sweep (RegularExpireStrategy.java:94-124): removes up to max_tokens
 * cached tokens (the reference: executeCount = 1000 per 1 s tick) and returns their counts to
 * nowCalls.  Which tokens go first when more than max_tokens are cached is unspecified (the
 * reference follows ConcurrentLinkedHashMap key order). */
int  sentinel_concurrent_expire(sentinel_engine_t *eng, int64_t max_tokens, int64_t *removed);

/* ---- per-call TokenService mirror (one event, synchronous) ---- */
int  sentinel_request_token(sentinel_engine_t *eng, int64_t flow_id, int32_t acquire_count,
                            int32_t prioritized, int64_t ts, sentinel_token_result_t *out);
int  sentinel_request_param_token(sentinel_engine_t *eng, int64_t flow_id, int32_t acquire_count,
                                  uint64_t param_key, int64_t ts, sentinel_token_result_t *out);

/* ---- concurrent per-call front door (TokenService contract under many threads) ----
 * Callers block in request_token; a dispatcher thread batches concurrent requests (up to
 * max_batch, or max_wait_us after the first) into one GPU batch in arrival order. */
typedef struct sentinel_batcher sentinel_batcher_t;
int  sentinel_batcher_create(sentinel_engine_t *eng, int32_t max_batch, int32_t max_wait_us, sentinel_batcher_t **out);
int  sentinel_batcher_destroy(sentinel_batcher_t *b);
int  sentinel_batcher_request_token(sentinel_batcher_t *b, int64_t flow_id, int32_t acquire_count,
                                    int32_t prioritized, int64_t ts, sentinel_token_result_t *out);
/* Asynchronous variant for event-loop front ends (a Netty handler that writes the response when the
 * verdict arrives, the native wire server): returns at once; cb(ctx, tag, result) runs on the
 * dispatcher thread once the request's batch is decided (it must not block). */
typedef void (*sentinel_token_cb)(void *ctx, uint64_t tag, const sentinel_token_result_t *result);
int  sentinel_batcher_request_token_async(sentinel_batcher_t *b, int64_t flow_id, int32_t acquire_count,
                                          int32_t prioritized, int64_t ts, sentinel_token_cb cb, void *ctx,
                                          uint64_t tag);
/* n asynchronous requests in one call (one lock round trip for a front end that decoded many frames
 * at once): request i is (flow_ids[i], acquire[i], prioritized ? prioritized[i] : 0, ts[i]) with
 * tag tags[i]. */
int  sentinel_batcher_request_tokens_async(sentinel_batcher_t *b, int32_t n, const int64_t *flow_ids,
                                           const int32_t *acquire, const uint8_t *prioritized, const int64_t *ts,
                                           sentinel_token_cb cb, void *ctx, const uint64_t *tags);
/* fn(ctx) runs on the dispatcher thread after the callbacks of every decided batch (a front end
 * flushes its sockets once per batch instead of once per response); NULL removes the hook. */
int  sentinel_batcher_set_batch_hook(sentinel_batcher_t *b, void (*fn)(void *ctx), void *ctx);
int  sentinel_batcher_stats(sentinel_batcher_t *b, int64_t *batches, int64_t *requests);

/* ---- native cluster token server (the reference's Netty transport over TCP) ----
 * The reference's framing and codecs (NettyTransportServer.java:89-92, DefaultRequestEntityDecoder,
 * Ping/Flow/ParamFlow request decoders, DefaultResponseEntityWriter) in front of one engine: epoll
 * I/O threads decode frames, FLOW requests go to an internal batcher (one call per socket read),
 * responses are flushed once per decided batch; PARAM requests of a read are one host batch; PINGs
 * maintain the namespace's connection set and connectedCount (ConnectionManager). */
typedef struct sentinel_param_interner sentinel_param_interner_t;
int  sentinel_param_interner_create(sentinel_param_interner_t **out);
int  sentinel_param_interner_destroy(sentinel_param_interner_t *it);
/* (flowId, Java-typed value) -> injective param key, dense from 1 (Java equals(): the type is part
 * of the key, NaNs canonical, strings by their decoded text).  `value` = the value's wire bytes after
 * its type byte (ParamFlowRequestDataWriter): big-endian int / long / short / byte / boolean / float
 * bits / double bits, or a string's UTF-8 bytes. */
int  sentinel_param_interner_key(sentinel_param_interner_t *it, int64_t flow_id, int32_t type, const uint8_t *value,
                                 int32_t len, uint64_t *key);
/* The same for a request at time ts (ms): the entry's last use.  The interner is bounded: past
 * max_entries (default 2^23) entries idle for more than idle_ms (default 60000) are forgotten --
 * exact when idle_ms >= every param rule's interval (such a value has no valid bucket left); if a
 * flood of distinct values inside that horizon still exceeds the cap, the least recently used go
 * (the reference bounds its CacheMaps by LRU, ConcurrentLinkedHashMapWrapper.java:35-43).  The wire
 * server interns only values of flowIds that have a param rule (others answer NO_RULE_EXISTS). */
int  sentinel_param_interner_key_at(sentinel_param_interner_t *it, int64_t flow_id, int32_t type, const uint8_t *value,
                                    int32_t len, int64_t ts, uint64_t *key);
int  sentinel_param_interner_set_limits(sentinel_param_interner_t *it, int64_t max_entries, int64_t idle_ms);
int  sentinel_param_interner_stats(sentinel_param_interner_t *it, int64_t *entries, int64_t *evicted);
/* Full passes over the map so far: each ends at or below 3/4 of max_entries, so a pass runs at most
 * once per max_entries / 4 new values (bounded work per insert under a steady flood of values). */
int  sentinel_param_interner_scans(sentinel_param_interner_t *it, int64_t *scans);
typedef int64_t (*sentinel_clock_fn)(void *ctx);
typedef struct {
    const char *host;                 /* IPv4 bind address, NULL = 127.0.0.1 */
    int32_t port;                     /* 0 = ephemeral (sentinel_wire_server_port) */
    int32_t io_threads;               /* epoll loops, >= 1 */
    int32_t max_batch, max_wait_us;   /* the internal batcher */
    const char *const *namespaces;    /* the engine's namespace table, in order (PING names) */
    int32_t n_namespaces;
    sentinel_param_interner_t *interner;   /* NULL: the server's own */
    sentinel_clock_fn clock;          /* NULL: wall-clock ms (TimeUtil.currentTimeMillis) */
    void *clock_ctx;
} sentinel_wire_config_t;
typedef struct sentinel_wire_server sentinel_wire_server_t;
int  sentinel_wire_server_create(sentinel_engine_t *eng, const sentinel_wire_config_t *cfg, sentinel_wire_server_t **out);
int32_t sentinel_wire_server_port(sentinel_wire_server_t *srv);
int  sentinel_wire_server_stats(sentinel_wire_server_t *srv, int64_t *flow_requests, int64_t *param_requests,
                                int64_t *batches, int32_t *connections);
int  sentinel_wire_server_destroy(sentinel_wire_server_t *srv);

/* ---- one node, several devices ----
 * One engine per entry of device_ids (a device may repeat: several shards on one GPU); flows are
 * partitioned shard = splitmix64(flowId) mod n (a flow's verdicts depend only on its own window and
 * host constants: no exchange on the decision path).  Rule tables are split by shard (the
 * putMetricIfAbsent orphan rule still sees the whole node's namespace lists); namespace and server
 * config are broadcast.  Replaces one DefaultTokenService over the whole flowId space.  The
 * GlobalRequestLimiter couples a namespace's flows, so sentinel_cluster_set_namespaces rejects
 * (SENTINEL_E_INVALID) any namespace with has_limiter when the cluster has more than one shard: each
 * shard would otherwise apply the full maxAllowedQps to its share and the node could admit up to
 * n x the cap.  Multi-GPU deployments with limiters shard by namespace instead (one process per GPU,
 * sentinel_amd/shard.py shard_by_namespace). */
typedef struct sentinel_cluster sentinel_cluster_t;
int32_t sentinel_shard_of(int64_t flow_id, int32_t n_shards);
int  sentinel_cluster_create(const int32_t *device_ids, int32_t n, const sentinel_server_config_t *cfg,
                             sentinel_cluster_t **out);
int  sentinel_cluster_destroy(sentinel_cluster_t *c);
int32_t sentinel_cluster_size(sentinel_cluster_t *c);
int  sentinel_cluster_engine(sentinel_cluster_t *c, int32_t shard, sentinel_engine_t **out);
int  sentinel_cluster_set_server_config(sentinel_cluster_t *c, const sentinel_server_config_t *cfg);
int  sentinel_cluster_set_namespaces(sentinel_cluster_t *c, const sentinel_namespace_t *ns, int32_t n);
int  sentinel_cluster_set_connected_count(sentinel_cluster_t *c, int32_t namespace_idx, int32_t connected);
int  sentinel_cluster_load_flow_rules(sentinel_cluster_t *c, const sentinel_flow_rule_t *rules, int32_t n);
int  sentinel_cluster_load_param_rules(sentinel_cluster_t *c, const sentinel_param_rule_t *rules, int32_t n,
                                       const uint64_t *hot_keys, const int32_t *hot_counts, int32_t n_hot);
/* requestToken for a host batch of flowIds (flags bit 0: prioritized): routed to the owning shards
 * (arrival order kept per flow), decided concurrently, verdicts at the arrival positions. */
int  sentinel_cluster_submit_host(sentinel_cluster_t *c, int64_t n, const int64_t *flow_ids, const int32_t *acquire,
                                  const int64_t *ts, const uint8_t *flags, sentinel_verdict_t *verdicts);
int32_t sentinel_cluster_flow_count(sentinel_cluster_t *c);
/* Every shard's snapshot records at ts, shard after shard; cap >= sentinel_cluster_flow_count. */
int  sentinel_cluster_snapshot(sentinel_cluster_t *c, int64_t ts, sentinel_flow_snapshot_t *out, int64_t cap,
                               int64_t *n_out);
/* The per-call front door over every shard: one batcher (dispatcher thread) per engine, each call
 * routed to its flow's shard. */
int  sentinel_cluster_batchers_create(sentinel_cluster_t *c, int32_t max_batch, int32_t max_wait_us);
int  sentinel_cluster_request_token(sentinel_cluster_t *c, int64_t flow_id, int32_t acquire_count,
                                    int32_t prioritized, int64_t ts, sentinel_token_result_t *out);

/* ---- observability / parity ---- */
int  sentinel_synchronize(sentinel_engine_t *eng);
/* Flow metric dump: sample_count x {window start ms (-1 = absent), 7 counters}, then 7 occupy
 * counters, then has_occupied (same layout as the oracle's orc_cm_dump). */
int  sentinel_dump_flow(sentinel_engine_t *eng, int32_t flow_idx, int64_t *out, int32_t out_len);
/* Sum of one param value's counters over the valid window at ts (ClusterParamMetric.getSum). */
int  sentinel_param_sum(sentinel_engine_t *eng, int32_t rule_idx, uint64_t param_key, int64_t ts, int64_t *out);
/* Snapshot of every loaded flow at ts: getAvg(BLOCK), getAvg(PASS) (each read rolls the window,
 * as the reference does).  out has sentinel_flow_count() entries (host memory). */
int  sentinel_snapshot(sentinel_engine_t *eng, int64_t ts, sentinel_flow_snapshot_t *out);
/* Device-pointer variant (for the RCCL all-gather), asynchronous on `stream`. */
int  sentinel_snapshot_device(sentinel_engine_t *eng, int64_t ts, sentinel_flow_snapshot_t *d_out, void *stream);

/* getTopValues(number) of every loaded param rule at ts (ClusterParamMetric.getTopValues,
 * sentinel-cluster/.../cluster/flow/statistic/metric/ClusterParamMetric.java:84-127): per rule up to
 * `number` (param key, avg = sum / intervalInSecond) with a non-zero window count, by (int) count
 * descending, equal (int) counts by key ascending (the reference leaves their order to HashMap
 * iteration).  count[r] entries for rule r; keys / avgs are rule-major [rules][number].  Exact mode
 * only (the count-min sketch keeps no keys: every count is 0).  Host pointers, synchronous. */
int  sentinel_param_top_values(sentinel_engine_t *eng, int64_t ts, int32_t number, int32_t *count,
                               uint64_t *keys, double *avgs);
/* ClusterMetricNodeGenerator.paramToMetricNode (ClusterMetricNodeGenerator.java:88-105) per param rule:
 * flowId + topParams = getTopValues(5), for the RCCL all-gather of the snapshot.  DEVICE pointer with
 * one record per loaded param rule; synchronous on `stream`. */
#define SENTINEL_TOP_PARAMS 5
typedef struct {
    int64_t  flow_id;
    int32_t  n_top;
    int32_t  reserved;
    uint64_t key[SENTINEL_TOP_PARAMS];
    double   avg[SENTINEL_TOP_PARAMS];
} sentinel_param_snapshot_t;
int  sentinel_param_snapshot_device(sentinel_engine_t *eng, int64_t ts, sentinel_param_snapshot_t *d_out, void *stream);

/* ---- metric registry (ClusterMetricStatistics / ClusterParamMetricStatistics) ---- */
/* The window {sampleCount, intervalMs} of the METRIC behind a flow: a reload keeps a surviving flowId's
 * metric as it was built (ClusterFlowRuleManager.java:361-362), so it can differ from its rule's. */
int  sentinel_flow_window(sentinel_engine_t *eng, int32_t flow_idx, int32_t *sample_count, int32_t *interval_ms);
/* ClusterMetricStatistics.METRIC_MAP.size(): flow metrics held, orphaned ones included. */
int64_t sentinel_metric_count(sentinel_engine_t *eng);
/* Server window change (ServerFlowConfig sampleCount / intervalMs; ClusterServerConfigManager.java:333-343):
 * ClusterMetricStatistics.resetFlowMetrics + ClusterParamMetricStatistics.resetFlowMetrics -- every flow and
 * param metric, orphans included, restarts empty with this window.  An invalid window is ignored. */
int  sentinel_reset_metrics(sentinel_engine_t *eng, int32_t sample_count, int32_t interval_ms);
/* Param slot table statistics: {capacity, live slots after the last rebuild, rebuilds so far}. */
int  sentinel_param_table_stats(sentinel_engine_t *eng, int64_t *out3);
/* Shared count-min sketch batches so far: {decided by the two-phase key walk, sent to the per-rule lanes
 * because one key-hash sub-range held more requests than one LDS chunk}. */
int  sentinel_param_cm_stats(sentinel_engine_t *eng, int64_t *out2);
/* ... of the key-walk batches, those decided by the block-owned walk (each sketch block staged in LDS by
 * one workgroup: k_pp_cm_block). */
int  sentinel_param_cm_block_batches(sentinel_engine_t *eng, int64_t *out);
/* Flow batches so far by pipeline: {small (one launch), sorted (radix sort), partition (prep + scan +
 * scatter), of the partition batches those with decide-order output (sentinel_submit_flow_batch_ordered)}. */
int  sentinel_flow_path_stats(sentinel_engine_t *eng, int64_t *out4);
/* The engine's own stream (hipStream_t). */
void *sentinel_engine_stream(sentinel_engine_t *eng);
/* Per-kernel timing with HIP events recorded on the launch stream (for roofline reporting).
 * enable=1 starts (and clears) the record, 0 stops.  profile_read synchronises, then fills up to
 * `max` entries: names (32 chars each), total milliseconds, launch count and events processed
 * (summed over launches); returns the number of entries. */
int  sentinel_profile_enable(sentinel_engine_t *eng, int enable);
/* Time only the named kernel (NULL or "": every kernel): two events per launch of it instead of two
 * per launch of every kernel, so a timed run keeps its dominant kernel's live duration cheaply. */
int  sentinel_profile_select(sentinel_engine_t *eng, const char *kernel);
/* Flow pipeline of the following batches: 0 auto (one launch for batches of <= 4096 events, else
 * partition-local for >= 32768 flows, radix sort after a skewed batch), 1 the global radix sort,
 * 2 the partition-local path, 3 the one-launch small-batch kernel over consecutive chunks of 4096
 * events (2 and 3 where they apply: no namespace limiter, <= 16 buckets).  Verdicts are identical
 * on every path. */
int  sentinel_set_flow_path(sentinel_engine_t *eng, int path);
/* Gate the timing of following launches on (1) or off (0) without collecting or clearing what was
 * timed so far (no host synchronisation: callable between the batches of a timed loop). */
int  sentinel_profile_gate(sentinel_engine_t *eng, int on);
/* With profiling on, time only every k-th launch of the selected kernel (default 1). */
int  sentinel_profile_every(sentinel_engine_t *eng, int every);
int  sentinel_profile_read(sentinel_engine_t *eng, int max, char *names32, double *total_ms,
                           int64_t *calls, int64_t *units);

#ifdef __cplusplus
}
#endif
#endif
