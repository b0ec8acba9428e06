"""Host side of the metric snapshots: formatting of the device's metric rows as the
reference's metrics.log lines and the cluster server's metricList.

  MetricNode.toFatString / toThinString   core/.../node/metric/MetricNode.java:150-229
  MetricWriter (one file per day)         core/.../node/metric/MetricWriter.java (size rolling and the .idx
                                          index file are not restated: lines are appended to
                                          {app}-metrics.log.{yyyy-MM-dd})
  ClusterMetricNodeGenerator.generateCurrentNodeMap
                                          srv/flow/statistic/ClusterMetricNodeGenerator.java:39-105

The rows themselves come from the device (sg_local_metrics, sg_snapshot_metrics, sg_cparam_top_values).
"""
import datetime
import os

import numpy as np

from . import abi


def _date(ts_ms, tz):
    return datetime.datetime.fromtimestamp(ts_ms / 1000.0, tz).strftime("%Y-%m-%d %H:%M:%S")


def fat_line(row, resource_name, classification=0, tz=datetime.timezone.utc):
    """MetricNode.toFatString: timestamp|yyyy-MM-dd HH:mm:ss|resource|pass|block|success|exception|rt|occupied|
    concurrency|classification, "|" in the name replaced by "_"."""
    name = resource_name.replace("|", "_")
    return (f"{int(row['timestamp'])}|{_date(int(row['timestamp']), tz)}|{name}|{int(row['pass_qps'])}|"
            f"{int(row['block_qps'])}|{int(row['success_qps'])}|{int(row['exception_qps'])}|{int(row['rt'])}|"
            f"{int(row['occupied_pass_qps'])}|{int(row['concurrency'])}|{classification}\n")


def thin_line(row, resource_name, classification=0):
    """MetricNode.toThinString."""
    name = resource_name.replace("|", "_")
    return (f"{int(row['timestamp'])}|{name}|{int(row['pass_qps'])}|{int(row['block_qps'])}|{int(row['success_qps'])}|"
            f"{int(row['exception_qps'])}|{int(row['rt'])}|{int(row['occupied_pass_qps'])}|{int(row['concurrency'])}|"
            f"{classification}")


def parse_fat_line(line):
    """MetricNode.fromFatString → dict."""
    s = line.rstrip("\n").split("|")
    out = {"timestamp": int(s[0]), "resource": s[2], "pass_qps": int(s[3]), "block_qps": int(s[4]),
           "success_qps": int(s[5]), "exception_qps": int(s[6]), "rt": int(s[7])}
    if len(s) >= 9:
        out["occupied_pass_qps"] = int(s[8])
    if len(s) >= 10:
        out["concurrency"] = int(s[9])
    if len(s) == 11:
        out["classification"] = int(s[10])
    return out


class MetricWriter:
    """MetricTimerListener's writer: rows grouped by timestamp (ascending), appended as fat lines to the day's
    file {base_dir}/{app}-metrics.log.{yyyy-MM-dd}."""

    def __init__(self, base_dir, app_name, resource_names, tz=datetime.timezone.utc):
        self.base_dir, self.app, self.names, self.tz = base_dir, app_name, resource_names, tz
        os.makedirs(base_dir, exist_ok=True)

    def path_for(self, ts_ms):
        day = datetime.datetime.fromtimestamp(ts_ms / 1000.0, self.tz).strftime("%Y-%m-%d")
        return os.path.join(self.base_dir, f"{self.app}-metrics.log.{day}")

    def write(self, rows):
        rows = np.asarray(rows, dtype=abi.METRIC_NODE_DTYPE)
        for r in rows:
            with open(self.path_for(int(r["timestamp"])), "a") as f:
                f.write(fat_line(r, self.names[int(r["resource"])], tz=self.tz))
        return len(rows)


def cluster_node_map(now_ms, flow_rules, flow_names, flow_snapshot, param_rules=None, param_names=None,
                     param_top=None):
    """ClusterMetricNodeGenerator.generateCurrentNodeMap for one namespace: resource name → [ClusterMetricNode].
    flow_snapshot: [K, 2] {passQps, blockQps} (sg_snapshot_metrics or the node-wide rollup); param_top: per cluster
    param rule the getTopValues(5) list [(value, qps), ...] (sg_cparam_top_values)."""
    out = {}
    for k, r in enumerate(flow_rules):
        node = {"timestamp": now_ms, "flowId": int(r["flow_id"]), "resourceName": flow_names[k],
                "passQps": float(flow_snapshot[k][0]), "blockQps": float(flow_snapshot[k][1]), "topParams": None}
        out.setdefault(flow_names[k], []).append(node)
    for k, r in enumerate(param_rules if param_rules is not None else []):
        node = {"timestamp": now_ms, "flowId": int(r["flow_id"]), "resourceName": param_names[k],
                "passQps": 0.0, "blockQps": 0.0, "topParams": dict(param_top[k])}
        out.setdefault(param_names[k], []).append(node)
    return out
