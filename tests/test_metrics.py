"""Metric snapshots on the CPU side: the oracle's StatisticNode.metrics() rows
(StatisticNode.java:116-147, ArrayMetric.details/fromBucket :156-204), ClusterParamMetric.getTopValues restating
ClusterParamMetricTest.testClusterParamMetric (sentinel-cluster-server-default/src/test/.../metric/
ClusterParamMetricTest.java:27-55), and the metrics.log line format (MetricNode.toFatString / fromFatString,
MetricNodeTest.testFromFatString)."""
import datetime

import numpy as np
import pytest

from oracle.binding import ClusterParamMetric, LocalChain, local_rule
from sentinel_amd import abi
from sentinel_amd.metrics import MetricWriter, fat_line, parse_fat_line, thin_line

T0 = 1_700_000_000_000  # a whole second


def test_cluster_param_metric_top_values():
    m = ClusterParamMetric(5, 25)
    e1, e2, e3 = 1, 2, 3
    t = T0 + 7
    for v, c in ((e1, -1), (e1, -2), (e2, 100), (e2, 23), (e3, 100), (e3, 230)):
        m.add_value(t, v, c)
    assert m.get_sum(t, e1) == -3 and m.get_avg(t, e1) == pytest.approx(-120, abs=0.01)
    assert m.top_values(t, 1) == {e3: 13200.0}
    assert m.top_values(t, 5) == {e3: 13200.0, e2: 4920.0, e1: -120.0}
    m.add_value(t, e2, 100)
    m.add_value(t, e2, 23)
    assert m.get_sum(t, e2) == 246 and m.get_avg(t, e2) == pytest.approx(9840, abs=0.01)
    with pytest.raises(ValueError):
        m.top_values(t, -1)


def test_statistic_node_metric_rows():
    ch = LocalChain()
    ch.load_rules(np.array([local_rule(), local_rule()]))
    # second 0: 3 passes + 2 exits (rt 10 and 30) on resource 0; second 1: 1 pass on resource 1; second 2: nothing
    ch.entry(T0 + 5)
    ch.entry(T0 + 6)
    ch.entry(T0 + 7, count=2)
    ch.exit(T0 + 15, T0 + 5)
    ch.exit(T0 + 36, T0 + 6, error=True)
    ch.entry(T0 + 1500, res=1)
    rows = ch.metrics(T0 + 1700)     # now's second (T0 + 1000) is not reported yet
    assert len(rows) == 1
    r = rows[0]
    assert (r["timestamp"], r["resource"], r["pass_qps"], r["success_qps"], r["exception_qps"], r["rt"]) == \
        (T0, 0, 4, 2, 1, 20)
    assert len(ch.metrics(T0 + 1800)) == 0                    # lastFetchTime: reported once
    rows = ch.metrics(T0 + 2100)
    assert [(int(x["timestamp"]), int(x["resource"]), int(x["pass_qps"])) for x in rows] == [(T0 + 1000, 1, 1)]
    assert len(ch.metrics(T0 + 70_000)) == 0


def test_fat_and_thin_lines(tmp_path):
    row = np.zeros((), abi.METRIC_NODE_DTYPE)
    row["timestamp"], row["pass_qps"], row["success_qps"], row["concurrency"] = 1564382218000, 1, 1, 2
    line = fat_line(row, "/foo/*", classification=1, tz=datetime.timezone(datetime.timedelta(hours=8)))
    assert line == "1564382218000|2019-07-29 14:36:58|/foo/*|1|0|1|0|0|0|2|1\n"   # MetricNodeTest's line
    p = parse_fat_line(line)
    assert p["classification"] == 1 and p["concurrency"] == 2 and p["success_qps"] == 1
    assert thin_line(row, "a|b") == "1564382218000|a_b|1|0|1|0|0|0|2|0"
    w = MetricWriter(str(tmp_path), "app", ["/foo/*"])
    assert w.write(np.array([row])) == 1
    assert open(w.path_for(1564382218000)).read().startswith("1564382218000|2019-07-29 06:36:58|/foo/*|1|")
