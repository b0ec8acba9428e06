"""Host side of the metric snapshots: formatting of the device's metric rows as the
reference's metrics.log lines and the cluster server's metricList.

  MetricNode.toFatString / toThinString   core/.../node/metric/MetricNode.java:150-229
  MetricWriter                            core/.../node/metric/MetricWriter.java: files
                                          {app}-metrics.log[.pid{pid}].{yyyy-MM-dd}[.n] rolled by size and day, the
                                          .idx index of (second, offset) pairs, the total-file-count cap
  MetricTimerListener.run                 core/.../node/metric/MetricTimerListener.java:40-69 (rows grouped by second,
                                          Constants.ENTRY_NODE's rows with the resources')
  MetricSearcher.find                     core/.../node/metric/MetricSearcher.java (the index lookup)
  ClusterMetricNodeGenerator.generateCurrentNodeMap
                                          srv/flow/statistic/ClusterMetricNodeGenerator.java:39-105

The rows themselves come from the device (sg_local_metrics, sg_snapshot_metrics, sg_cparam_top_values).
"""
import datetime
import os
import re
import struct

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


ENTRY_NODE_NAME = "__total_inbound_traffic__"  # Constants.TOTAL_IN_RESOURCE_NAME
METRIC_FILE = "metrics.log"
METRIC_FILE_INDEX_SUFFIX = ".idx"


def form_metric_file_name(app_name, pid=None):
    """MetricWriter.formMetricFileName (:376-395): '.' in the app name becomes '-'; '.pid{pid}' when the log name
    uses the pid (LogBase.isLogNameUsePid)."""
    app = (app_name or "").replace(".", "-")
    name = app + "-" + METRIC_FILE
    if pid is not None:
        name += f".pid{pid}"
    return name


def form_index_file_name(metric_file_name):
    return metric_file_name + METRIC_FILE_INDEX_SUFFIX


def _file_name_key(path):
    """METRIC_FILE_NAME_CMP (:245-280): date part (skipping a pid part), then name length, then the name."""
    name = os.path.basename(path)
    parts = name.split(".")
    date = parts[2]
    if date.startswith("pid"):
        date = parts[3]
    return (date, len(name), name)


def sort_metric_file_names(names):
    return sorted(names, key=_file_name_key)


def file_name_matches(file_name, base_file_name):
    """MetricWriter.fileNameMatches (:320-331): base + '.yyyy-MM-dd' + optional '.number'."""
    if not file_name.startswith(base_file_name):
        return False
    return re.fullmatch(r"\.[0-9]{4}-[0-9]{2}-[0-9]{2}(\.[0-9]*)?", file_name[len(base_file_name):]) is not None


def list_metric_files(base_dir, base_file_name):
    """MetricWriter.listMetricFiles (:296-318): matching metric files (not .idx / .lck), sorted."""
    out = []
    for fn in os.listdir(base_dir):
        p = os.path.join(base_dir, fn)
        if (os.path.isfile(p) and file_name_matches(fn, base_file_name) and not fn.endswith(METRIC_FILE_INDEX_SUFFIX)
                and not fn.endswith(".lck")):
            out.append(os.path.abspath(p))
    return sort_metric_file_names(out)


class MetricWriter:
    """MetricWriter (core/.../node/metric/MetricWriter.java) over a given clock and time zone: write(time, nodes)
    appends one second's rows as fat lines to the current file through a buffered stream and, when the second
    advances, first records (second, offset) in the .idx file (big-endian longs, DataOutputStream.writeLong); a
    file that reached single_file_size or a new day starts the next file of the day
    ({base}.{yyyy-MM-dd}[.n], nextFileNameOfDay), keeping at most total_file_count files (removeMoreFiles).
    start_ms is the construction time (lastSecond starts there, as System.currentTimeMillis() in the constructor)."""

    def __init__(self, base_dir, app_name, single_file_size, total_file_count=6, pid=None, start_ms=0,
                 tz=datetime.timezone.utc, resource_names=None, classifications=None):
        if single_file_size <= 0 or total_file_count <= 0:
            raise ValueError("singleFileSize and totalFileCount must be > 0")
        self.base_dir = base_dir
        os.makedirs(base_dir, exist_ok=True)
        self.app, self.pid, self.tz = app_name, pid, tz
        # MetricWriter.timeSecondBase: "1970-01-01 00:00:00" parsed in the writer's zone = -(the zone's offset then)
        self._epoch_off = int(datetime.datetime(1970, 1, 1, tzinfo=tz).utcoffset().total_seconds())
        self.single_file_size, self.total_file_count = single_file_size, total_file_count
        self.last_second = start_ms // 1000
        self.base_file_name = None
        self.cur_file = self.cur_index = None
        self._out = self._idx = None
        self.names = resource_names
        self.classifications = classifications

    # -- file handling (closeAndNewFile :349-365, nextFileNameOfDay :190-214, removeMoreFiles :333-347)
    def _next_file_name_of_day(self, time_ms):
        date = datetime.datetime.fromtimestamp(time_ms / 1000.0, self.tz).strftime("%Y-%m-%d")
        model = f"{self.base_file_name}.{date}"
        found = [os.path.join(self.base_dir, fn) for fn in os.listdir(self.base_dir)
                 if model in fn and not fn.endswith(METRIC_FILE_INDEX_SUFFIX) and not fn.endswith(".lck")]
        if not found:
            return os.path.join(self.base_dir, model)
        last = sort_metric_file_names(found)[-1]
        tail = last.split(".")[-1]
        n = int(tail) if re.fullmatch(r"[0-9]{1,10}", tail) else 0
        return os.path.join(self.base_dir, f"{model}.{n + 1}")

    def _remove_more_files(self):
        files = list_metric_files(self.base_dir, self.base_file_name)
        for fn in files[:max(0, len(files) - self.total_file_count + 1)]:
            for p in (fn, form_index_file_name(fn)):
                if os.path.exists(p):
                    os.remove(p)

    def _close_and_new_file(self, path):
        self._remove_more_files()
        self.close()
        self._out = open(path, "wb")              # FileOutputStream(fileName, append = false)
        self._idx = open(form_index_file_name(path), "wb")
        self.cur_file, self.cur_index = path, form_index_file_name(path)

    def _valid_size(self):
        return os.path.getsize(self.cur_file) < self.single_file_size

    def _is_new_day(self, last_second, second):
        # MetricWriter.isNewDay: (second - timeSecondBase) / 86400 with one timeSecondBase, "1970-01-01 00:00:00"
        # parsed in the writer's zone once (the zone's offset at the epoch, not at either second)
        return (second + self._epoch_off) // 86400 > (last_second + self._epoch_off) // 86400

    def _write_lines(self, nodes):
        buf = "".join(fat_line(r, self._name(r), self._cls(r), tz=self.tz) for r in nodes).encode("utf-8")
        self._out.write(buf)
        self._out.flush()

    def _name(self, r):
        res = int(r["resource"])
        if res == abi.ENTRY_NODE_RESOURCE:
            return ENTRY_NODE_NAME
        return self.names[res] if self.names is not None else str(res)

    def _cls(self, r):
        res = int(r["resource"])
        if self.classifications is None or res == abi.ENTRY_NODE_RESOURCE:
            return 0
        return int(self.classifications[res])

    def write(self, time_ms, nodes):
        """MetricWriter.write(time, nodes) (:121-174): every node's timestamp becomes time_ms."""
        nodes = np.array(nodes, dtype=abi.METRIC_NODE_DTYPE, copy=True)
        nodes["timestamp"] = time_ms
        if self.cur_file is None:
            self.base_file_name = form_metric_file_name(self.app, self.pid)
            self._close_and_new_file(self._next_file_name_of_day(time_ms))
        if not (os.path.exists(self.cur_file) and os.path.exists(self.cur_index)):
            self._close_and_new_file(self._next_file_name_of_day(time_ms))
        second = time_ms // 1000
        if second < self.last_second:
            return  # earlier than the last second written: ignored (should not happen)
        if second > self.last_second:
            self._idx.write(struct.pack(">qq", second, self._out.tell()))   # writeIndex(second, position)
            self._idx.flush()
            if self._is_new_day(self.last_second, second):
                self._close_and_new_file(self._next_file_name_of_day(time_ms))
            self.last_second = second
        self._write_lines(nodes)
        if not self._valid_size():
            self._close_and_new_file(self._next_file_name_of_day(time_ms))

    def close(self):
        for f in (self._out, self._idx):
            if f is not None:
                f.close()
        self._out = self._idx = None


class MetricTimerListener:
    """MetricTimerListener.run (:40-55) over the device rows of one sg_local_metrics call (ENTRY_NODE rows included,
    resource = abi.ENTRY_NODE_RESOURCE): rows grouped by timestamp in ascending order, one write per second."""

    def __init__(self, writer):
        self.writer = writer

    def run(self, rows):
        rows = np.asarray(rows, dtype=abi.METRIC_NODE_DTYPE)
        if len(rows) == 0:
            return 0
        order = np.lexsort((rows["resource"], rows["resource"] == abi.ENTRY_NODE_RESOURCE, rows["timestamp"]))
        rows = rows[order]
        ts = rows["timestamp"]
        cut = np.nonzero(np.diff(ts))[0] + 1
        for part in np.split(rows, cut):
            self.writer.write(int(part["timestamp"][0]), part)
        return len(rows)


def read_index(index_file):
    """The (second, offset) pairs of a .idx file."""
    with open(index_file, "rb") as f:
        data = f.read()
    return [struct.unpack(">qq", data[i:i + 16]) for i in range(0, len(data) - len(data) % 16, 16)]


def find(base_dir, base_file_name, begin_ms, recommend_lines):
    """MetricSearcher.find (:78-99) without the cached position: the first file whose index has a second >= begin,
    then fat lines from that offset on (across the following files), whole seconds, about recommend_lines."""
    files = list_metric_files(base_dir, base_file_name)
    begin_s = begin_ms // 1000
    for i, fn in enumerate(files):
        offset = next((off for sec, off in read_index(form_index_file_name(fn)) if sec >= begin_s), -1)
        if offset == -1:
            continue
        out, last_sec = [], None
        for j in range(i, len(files)):
            with open(files[j], "rb") as f:
                f.seek(offset if j == i else 0)
                for line in f.read().decode("utf-8").splitlines():
                    node = parse_fat_line(line)
                    sec = node["timestamp"] // 1000
                    if len(out) >= recommend_lines and sec != last_sec:
                        return out
                    out.append(node)
                    last_sec = sec
        return out
    return None


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
