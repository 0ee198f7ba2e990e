/*
 * kwok_metrics.h — native Metric CR compiler (host C++, no GPU): a kwok Metric CR -> the device
 * programs kwk_metrics_load / kwk_histograms_load take (kwok_engine.h).  The drop-in for the
 * reference's per-scrape CEL compilation of Metric values, called from Go through cgo
 * (INTEGRATION.md):
 *
 *   reference (Go)                                              replaced by
 *   ----------------------------------------------------------  -----------------------------------
 *   UpdateHandler.updateGauge / updateCounter / updateHistogram  kwk_compile_metrics once per Metric
 *     -> h.environment.Compile(metricConfig.Value) per metric      CR -> kwk_metric_set_programs /
 *     and bucket  pkg/kwok/metrics/metrics.go:168-462              _histograms -> kwk_metrics_load /
 *   cel.Environment.Compile (cached by source)                     kwk_histograms_load; per scrape
 *     pkg/utils/cel/environment.go:98-114                          kwk_metrics_eval /
 *   the metrics environment (Usage / CumulativeUsage /             kwk_histograms_eval
 *     StartedContainersTotal, node / pod / container variables)
 *     pkg/kwok/metrics/evaluator.go:51-144,201-233
 *
 * A value lowers to a postfix program over doubles when it is double arithmetic over the
 * per-series inputs (KWK_MIN_*) and constants; constant sub-expressions are folded with CEL's
 * semantics (int / uint overflow, Quantity arithmetic incl. the Quantity x double x10 rule).  A
 * metric with any value that has no device form is reported in describe's "host_metrics": the
 * host evaluates it per series (its device program is a placeholder: NaN for a gauge / counter,
 * 0 for every bucket of a histogram), exactly as the Python host's MetricsProgram does
 * (kwok_amd/host/metrics.py, cel.py lower), which is this compiler's CPU cross-check: byte-equal
 * programs on the shipped Metric CR, the histogram CRs and the reference-vector CR
 * (tests/test_metric_compiler.py).  Labels stay host CEL (string-valued: Prometheus exposition).
 *
 * Threading: a metric set is read-only after kwk_compile_metrics; sets are independent.
 */
#ifndef KWOK_METRICS_H
#define KWOK_METRICS_H

#include <stdint.h>

#include "kwok_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

#define KWK_ENOLOWER (-5) /* kwk_cel_lower: a valid expression with no device form (host-evaluated) */

typedef struct kwk_metric_set kwk_metric_set;

/* message of the calling thread's last failing call (m may be NULL: the messages are kept per
 * thread, whichever set the call named) */
const char* kwk_metric_set_last_error(const kwk_metric_set* m);

/* metric_json: one v1alpha1 Metric object (JSON; {"kind": "Metric", "spec": {"path", "metrics":
 * [{name, help, kind: gauge|counter|histogram, dimension: node|pod|container (default node),
 * value, labels: [{name, value}], buckets: [{le, value, hidden}]}]}}).  KWK_EINVAL for a malformed
 * CR, an unknown kind / dimension, a histogram without buckets, or a value that does not compile
 * (CEL syntax, or a constant sub-expression whose evaluation fails: the reference's
 * EvaluateFloat64 would fail at every scrape). */
kwk_status kwk_compile_metrics(const char* metric_json, kwk_metric_set** out);
kwk_status kwk_metric_set_destroy(kwk_metric_set* m);

/* gauges and counters, in CR order (arrays owned by the set): for kwk_metrics_load */
kwk_status kwk_metric_set_programs(const kwk_metric_set* m, uint32_t* n_metrics, const kwk_metric_desc** metrics,
                                   uint32_t* n_ops, const kwk_metric_op** ops);
/* histograms, in CR order: for kwk_histograms_load */
kwk_status kwk_metric_set_histograms(const kwk_metric_set* m, uint32_t* n_hist, const kwk_histogram_desc** hists,
                                     uint32_t* n_buckets, const kwk_metric_bucket** buckets, uint32_t* n_ops,
                                     const kwk_metric_op** ops);
/* JSON owned by the set: {"path", "metrics": [{"name", "help", "kind", "dimension", "labels":
 * [{"name", "value"}], "device": bool, "reason": "...", "program": index among the gauges /
 * counters or among the histograms}], "host_metrics": [names]} */
kwk_status kwk_metric_set_describe(const kwk_metric_set* m, const char** json);

/* one value expression -> its device program (dimension KWK_METRIC_DIM_*, or 3 for a dimension
 * the Metric CRD does not define); *n_ops = the program length (also when cap is too small:
 * KWK_ECAP).  KWK_ENOLOWER: no device form; KWK_EINVAL: the expression does not compile. */
kwk_status kwk_cel_lower(const char* expr, uint32_t dimension, kwk_metric_op* out, uint32_t cap, uint32_t* n_ops);

#ifdef __cplusplus
}
#endif
#endif /* KWOK_METRICS_H */
