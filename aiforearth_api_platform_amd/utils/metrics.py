"""In-process metrics registry: counters, gauges, histograms -> Prometheus text + JSON.

Replaces App-Insights ``TrackMetric`` (``ProcessManager/Libraries/AppInsightsLogger.cs:84-90``)
and keeps the reference's metric *names*:

* ``CURRENT_REQUESTS/<cluster><apiPath>`` concurrent-request gauges
  (``RequestReporter/CurrentProcessingUpsert.cs:102-104``), the HPA scaling signal
  (``APIs/Charts/templates/appinsights-metric.yaml:1-7``);
* ``<EndpointPath>_<state>`` queue lengths (``Libraries/QueueLogger.cs:21-47``).

Per-GPU additions: batch-size histogram, images/s, HBM used, kernel time.
"""
from __future__ import annotations

import bisect
import math
import re
import threading
from typing import Dict, List, Optional, Sequence


class Counter:
    def __init__(self, name: str, help: str = ""):
        self.name, self.help = name, help
        self._v = 0.0
        self._mu = threading.Lock()

    def inc(self, v: float = 1.0) -> None:
        with self._mu:
            self._v += v

    @property
    def value(self) -> float:
        return self._v


class Gauge:
    def __init__(self, name: str, help: str = ""):
        self.name, self.help = name, help
        self._v = 0.0
        self._mu = threading.Lock()

    def set(self, v: float) -> None:
        self._v = float(v)

    def inc(self, v: float = 1.0) -> None:
        with self._mu:
            self._v += v

    def dec(self, v: float = 1.0) -> None:
        with self._mu:
            self._v -= v

    @property
    def value(self) -> float:
        return self._v


DEFAULT_BUCKETS = (0.0005, 0.001, 0.002, 0.005, 0.01, 0.02, 0.05, 0.1, 0.2, 0.5, 1.0, 2.0, 5.0, 10.0, 30.0)


class Histogram:
    """Fixed-bucket histogram plus a bounded reservoir for exact-ish percentiles."""

    def __init__(self, name: str, help: str = "", buckets: Sequence[float] = DEFAULT_BUCKETS,
                 reservoir: int = 65536):
        self.name, self.help = name, help
        self.buckets = tuple(sorted(buckets))
        self.counts = [0] * (len(self.buckets) + 1)
        self.sum = 0.0
        self.count = 0
        self._res: List[float] = []
        self._res_cap = reservoir
        self._res_i = 0
        self._mu = threading.Lock()

    def observe(self, v: float) -> None:
        with self._mu:
            self.counts[bisect.bisect_left(self.buckets, v)] += 1
            self.sum += v
            self.count += 1
            if len(self._res) < self._res_cap:
                self._res.append(v)
            else:
                self._res[self._res_i % self._res_cap] = v
                self._res_i += 1

    def observe_many(self, vs) -> None:
        for v in vs:
            self.observe(float(v))

    def percentile(self, q: float) -> float:
        with self._mu:
            if not self._res:
                return float("nan")
            s = sorted(self._res)
        return percentile(s, q)

    def reset(self) -> None:
        with self._mu:
            self.counts = [0] * (len(self.buckets) + 1)
            self.sum = 0.0
            self.count = 0
            self._res.clear()
            self._res_i = 0


def percentile(sorted_vals: Sequence[float], q: float) -> float:
    """Linear-interpolated percentile (numpy 'linear') of an ascending sequence, q in [0,100]."""
    if not sorted_vals:
        return float("nan")
    k = (len(sorted_vals) - 1) * q / 100.0
    f, c = math.floor(k), math.ceil(k)
    if f == c:
        return float(sorted_vals[int(k)])
    return float(sorted_vals[f] + (sorted_vals[c] - sorted_vals[f]) * (k - f))


_PROM_BAD = re.compile(r"[^a-zA-Z0-9_:]")


def prom_name(name: str) -> str:
    n = _PROM_BAD.sub("_", name)
    return n if not n[:1].isdigit() else "_" + n


class Registry:
    def __init__(self):
        self._mu = threading.Lock()
        self.counters: Dict[str, Counter] = {}
        self.gauges: Dict[str, Gauge] = {}
        self.histograms: Dict[str, Histogram] = {}

    def counter(self, name: str, help: str = "") -> Counter:
        with self._mu:
            c = self.counters.get(name)
            if c is None:
                c = self.counters[name] = Counter(name, help)
            return c

    def gauge(self, name: str, help: str = "") -> Gauge:
        with self._mu:
            g = self.gauges.get(name)
            if g is None:
                g = self.gauges[name] = Gauge(name, help)
            return g

    def histogram(self, name: str, help: str = "", buckets: Optional[Sequence[float]] = None) -> Histogram:
        with self._mu:
            h = self.histograms.get(name)
            if h is None:
                h = self.histograms[name] = Histogram(name, help, buckets or DEFAULT_BUCKETS)
            return h

    def snapshot(self) -> dict:
        with self._mu:
            cs, gs, hs = dict(self.counters), dict(self.gauges), dict(self.histograms)
        return {
            "counters": {k: v.value for k, v in cs.items()},
            "gauges": {k: v.value for k, v in gs.items()},
            "histograms": {k: {"count": h.count, "sum": h.sum, "p50": h.percentile(50), "p99": h.percentile(99)}
                           for k, h in hs.items()},
        }

    def prometheus_text(self) -> str:
        """Prometheus exposition format; original names kept in a ``name`` label."""
        with self._mu:
            cs, gs, hs = dict(self.counters), dict(self.gauges), dict(self.histograms)
        lines: List[str] = []
        for k, c in sorted(cs.items()):
            n = prom_name(k)
            lines += [f"# TYPE {n} counter", f'{n}{{name="{k}"}} {c.value}']
        for k, g in sorted(gs.items()):
            n = prom_name(k)
            lines += [f"# TYPE {n} gauge", f'{n}{{name="{k}"}} {g.value}']
        for k, h in sorted(hs.items()):
            n = prom_name(k)
            lines.append(f"# TYPE {n} histogram")
            acc = 0
            for b, cnt in zip(h.buckets, h.counts):
                acc += cnt
                lines.append(f'{n}_bucket{{le="{b}"}} {acc}')
            lines.append(f'{n}_bucket{{le="+Inf"}} {h.count}')
            lines.append(f"{n}_sum {h.sum}")
            lines.append(f"{n}_count {h.count}")
        return "\n".join(lines) + "\n"

    def clear(self) -> None:
        with self._mu:
            self.counters.clear()
            self.gauges.clear()
            self.histograms.clear()


REGISTRY = Registry()


def current_requests_key(cluster: str, api_path: str) -> str:
    """Key layout of the writer, CurrentProcessingUpsert.cs:102 ("CURRENT_REQUESTS/" + cluster + path).

    The reference reader (CurrentProcessingGet.cs:60) used a mismatching layout (Appendix B #8); we
    use this single layout for both directions.
    """
    return f"CURRENT_REQUESTS/{cluster}{api_path}"
