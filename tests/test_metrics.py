"""Metric snapshots on the CPU side: the oracle's StatisticNode.metrics() rows
(StatisticNode.java:116-147, ArrayMetric.details/fromBucket :156-204), ClusterParamMetric.getTopValues restating
ClusterParamMetricTest.testClusterParamMetric (sentinel-cluster-server-default/src/test/.../metric/
ClusterParamMetricTest.java:27-55), and the metrics.log line format (MetricNode.toFatString / fromFatString,
MetricNodeTest.testFromFatString), and MetricWriter's files (MetricWriterTest.testFileNameCmp / testFileNamePidCmp /
testFileNameMatches, sentinel-core/src/test/.../node/metric/MetricWriterTest.java:17-80; the index, rolling and
file-count behaviour traced from MetricWriter.java:120-216,321-363)."""
import datetime

import numpy as np
import pytest

from oracle.binding import ClusterParamMetric, LocalChain, local_rule
from sentinel_amd import abi
import os

from sentinel_amd import metrics as M
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
    w = MetricWriter(str(tmp_path), "app", 1 << 20, start_ms=1564382217000, resource_names=["/foo/*"],
                     classifications=[1])
    w.write(1564382218000, np.array([row]))
    w.close()
    f = M.list_metric_files(str(tmp_path), "app-metrics.log")
    assert [os.path.basename(x) for x in f] == ["app-metrics.log.2019-07-29"]
    assert open(f[0]).read() == "1564382218000|2019-07-29 06:36:58|/foo/*|1|0|1|0|0|0|2|1\n"


def test_file_name_cmp():
    arr = ["metrics.log.2018-03-06", "metrics.log.2018-03-07", "metrics.log.2018-03-07.51",
           "metrics.log.2018-03-07.10", "metrics.log.2018-03-06.100"]
    assert M.sort_metric_file_names(arr) == ["metrics.log.2018-03-06", "metrics.log.2018-03-06.100",
                                             "metrics.log.2018-03-07", "metrics.log.2018-03-07.10",
                                             "metrics.log.2018-03-07.51"]


def test_file_name_pid_cmp():
    arr = ["metrics.log.pid1234.2018-03-06", "metrics.log.pid1234.2018-03-07", "metrics.log.pid1234.2018-03-07.51",
           "metrics.log.pid1234.2018-03-07.10", "metrics.log.pid1234.2018-03-06.100"]
    assert M.sort_metric_file_names(arr) == [
        "metrics.log.pid1234.2018-03-06", "metrics.log.pid1234.2018-03-06.100", "metrics.log.pid1234.2018-03-07",
        "metrics.log.pid1234.2018-03-07.10", "metrics.log.pid1234.2018-03-07.51"]


def test_file_name_matches():
    assert M.file_name_matches("Sentinel-SDK-Demo-metrics.log.2018-03-06", "Sentinel-SDK-Demo-metrics.log")
    assert M.file_name_matches("Sentinel-Admin-metrics.log.pid22568.2018-12-24", "Sentinel-Admin-metrics.log.pid22568")
    assert M.file_name_matches("Sentinel-SDK-Demo-metrics.log.2018-03-06.11", "Sentinel-SDK-Demo-metrics.log")
    assert not M.file_name_matches("Sentinel-SDK-Demo-metrics.log.XXX.2018-03-06.11", "Sentinel-SDK-Demo-metrics.log")
    assert not M.file_name_matches("Sentinel-SDK-Demo-metrics.log.2018-03-06.11XXX", "Sentinel-SDK-Demo-metrics.log")
    assert M.form_metric_file_name("Sentinel.SDK.Demo") == "Sentinel-SDK-Demo-metrics.log"
    assert M.form_metric_file_name("Sentinel-Admin", pid=22568) == "Sentinel-Admin-metrics.log.pid22568"


def _rows(ts, resources):
    r = np.zeros(len(resources), abi.METRIC_NODE_DTYPE)
    r["timestamp"], r["resource"], r["pass_qps"] = ts, resources, 1
    return r


def test_writer_index_rolling_and_file_count(tmp_path):
    """The index holds (second, offset) for every second after the first; the same second appends without an index
    entry; a file over singleFileSize rolls to '.1', '.2'...; a new day starts '{date}' again; at most totalFileCount
    files (and their .idx) are kept; the searcher finds a second through the index."""
    d = str(tmp_path)
    t0 = 1_700_000_000_000          # 2023-11-14 22:13:20 UTC
    w = MetricWriter(d, "app", 250, total_file_count=3, pid=7, start_ms=t0, resource_names=["a", "b", "c"])
    base = "app-metrics.log.pid7"
    w.write(t0, _rows(t0, [0, 1]))                      # lastSecond == t0's second: no index entry
    first = w.cur_file
    assert M.read_index(M.form_index_file_name(first)) == []
    w.write(t0 + 1000, _rows(t0 + 1000, [2]))
    size1 = os.path.getsize(first)
    assert M.read_index(M.form_index_file_name(first)) == [((t0 + 1000) // 1000, size1 - len(
        fat_line(_rows(t0 + 1000, [2])[0], "c")))]
    for k in range(2, 6):                               # ~65 bytes a line: rolls past 250 bytes
        w.write(t0 + 1000 * k, _rows(t0 + 1000 * k, [0]))
    names = [os.path.basename(x) for x in M.list_metric_files(d, base)]
    assert names[0] == base + ".2023-11-14" and names[1] == base + ".2023-11-14.1"
    day2 = t0 + 86_400_000
    w.write(day2, _rows(day2, [1]))
    w.write(day2 + 86_400_000, _rows(day2 + 86_400_000, [1]))
    w.close()
    names = [os.path.basename(x) for x in M.list_metric_files(d, base)]
    assert len(names) <= 3 and names[-1] == base + ".2023-11-16" and names[-2] == base + ".2023-11-15"
    for n in names:
        assert os.path.exists(os.path.join(d, n + ".idx"))
    assert not [fn for fn in os.listdir(d) if fn.endswith(".idx") and fn[:-4] not in names]
    got = M.find(d, base, day2, 1)
    assert got[0]["timestamp"] == day2 and got[0]["resource"] == "b"


def test_timer_listener_groups_by_second_entry_node_last(tmp_path):
    d = str(tmp_path)
    t0 = 1_700_000_000_000
    w = MetricWriter(d, "app", 1 << 20, start_ms=t0 - 5000, resource_names=["a", "b"])
    rows = np.concatenate([_rows(t0 + 1000, [abi.ENTRY_NODE_RESOURCE, 1]), _rows(t0, [1, abi.ENTRY_NODE_RESOURCE, 0])])
    assert M.MetricTimerListener(w).run(rows) == 5
    w.close()
    f = M.list_metric_files(d, "app-metrics.log")[0]
    lines = [parse_fat_line(x) for x in open(f).read().splitlines()]
    assert [(x["timestamp"] - t0, x["resource"]) for x in lines] == [
        (0, "a"), (0, "b"), (0, M.ENTRY_NODE_NAME), (1000, "b"), (1000, M.ENTRY_NODE_NAME)]
    idx = M.read_index(M.form_index_file_name(f))
    assert [s for s, _ in idx] == [t0 // 1000, t0 // 1000 + 1]
    assert idx[0][1] == 0 and idx[1][1] == sum(len(fat_line(_rows(t0, [0])[0], n)) for n in ("a", "b", M.ENTRY_NODE_NAME))


def test_new_day_uses_the_epoch_offset_of_the_zone(tmp_path):
    """MetricWriter.isNewDay divides (second - timeSecondBase) by 86400 with timeSecondBase = "1970-01-01 00:00:00"
    parsed once in the writer's zone: in America/New_York (EST at the epoch) the day rolls at 05:00 UTC all year,
    i.e. at 01:00 local time under daylight saving time."""
    import datetime
    import zoneinfo
    tz = zoneinfo.ZoneInfo("America/New_York")
    w = MetricWriter(str(tmp_path), "app", 1 << 20, tz=tz)
    utc = datetime.timezone.utc
    s = lambda h, m: int(datetime.datetime(2024, 7, 1, h, m, tzinfo=utc).timestamp())  # noqa: E731
    assert not w._is_new_day(s(4, 10), s(4, 50))   # 00:10 → 00:50 EDT: the EST day has not rolled yet
    assert w._is_new_day(s(4, 50), s(5, 10))       # 00:50 → 01:10 EDT: 00:00 EST passed
    w.close()
