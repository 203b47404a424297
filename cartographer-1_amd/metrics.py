"""Metrics and score histograms of the constraint-builder drop-ins (Python
mirror of ``include/cartographer_amd/metrics.h``).

* ``Counter``, ``Gauge``, ``Histogram``, ``Family``, ``FamilyFactory``: the
  interfaces of the reference's ``cartographer/metrics`` (counter.h, gauge.h,
  histogram.h, family_factory.h), with ``Null`` instances and
  ``Histogram.FixedWidth`` / ``ScaledPowersOf`` (metrics/histogram.cc:39-62).
* ``InMemoryFamilyFactory``: keeps the values in memory (tests; callers
  without an exporter).
* ``ScoreHistogram``: ``common::Histogram`` (common/histogram.cc:27-75) in
  float32 arithmetic, ``ToString`` formatted as absl prints it.
"""

from __future__ import annotations

import bisect
import threading
from typing import Dict, List, Tuple

import numpy as np


class Counter:
    _null = None

    @classmethod
    def Null(cls) -> "Counter":
        if cls._null is None:
            cls._null = _NullCounter()
        return cls._null

    def Increment(self, by_value: float = 1.0):
        raise NotImplementedError


class Gauge:
    _null = None

    @classmethod
    def Null(cls) -> "Gauge":
        if cls._null is None:
            cls._null = _NullGauge()
        return cls._null

    def Increment(self, by_value: float = 1.0):
        raise NotImplementedError

    def Decrement(self, by_value: float = 1.0):
        raise NotImplementedError

    def Set(self, value: float):
        raise NotImplementedError


class Histogram:
    _null = None

    @classmethod
    def Null(cls) -> "Histogram":
        if cls._null is None:
            cls._null = _NullHistogram()
        return cls._null

    @staticmethod
    def FixedWidth(width: float, num_finite_buckets: int) -> List[float]:
        out, boundary = [], 0.0
        for _ in range(num_finite_buckets):
            boundary += width
            out.append(boundary)
        return out

    @staticmethod
    def ScaledPowersOf(base: float, scale_factor: float, max_value: float) -> List[float]:
        if not (base > 1 and scale_factor > 0):
            raise ValueError("base must be > 1 and scale_factor > 0")
        out, boundary = [], scale_factor
        while boundary < max_value:
            out.append(boundary)
            boundary *= base
        return out

    def Observe(self, value: float):
        raise NotImplementedError


class _NullCounter(Counter):
    def Increment(self, by_value: float = 1.0):
        pass


class _NullGauge(Gauge):
    def Increment(self, by_value: float = 1.0):
        pass

    def Decrement(self, by_value: float = 1.0):
        pass

    def Set(self, value: float):
        pass


class _NullHistogram(Histogram):
    def Observe(self, value: float):
        pass


class Family:
    def Add(self, labels: Dict[str, str]):
        raise NotImplementedError


class FamilyFactory:
    def NewCounterFamily(self, name: str, description: str) -> Family:
        raise NotImplementedError

    def NewGaugeFamily(self, name: str, description: str) -> Family:
        raise NotImplementedError

    def NewHistogramFamily(self, name: str, description: str, boundaries) -> Family:
        raise NotImplementedError


# ---- in-memory implementation ---------------------------------------------
class ValueCounter(Counter):
    def __init__(self):
        self.value = 0.0
        self._lock = threading.Lock()

    def Increment(self, by_value: float = 1.0):
        with self._lock:
            self.value += by_value


class ValueGauge(Gauge):
    def __init__(self):
        self.value = 0.0
        self._lock = threading.Lock()

    def Increment(self, by_value: float = 1.0):
        with self._lock:
            self.value += by_value

    def Decrement(self, by_value: float = 1.0):
        with self._lock:
            self.value -= by_value

    def Set(self, value: float):
        with self._lock:
            self.value = float(value)


class BucketHistogram(Histogram):
    """Prometheus semantics: bucket k counts observations <= boundaries[k]
    above the previous boundary; the last bucket (+Inf) the rest."""

    def __init__(self, boundaries):
        self.boundaries = list(boundaries)
        self.counts = [0] * (len(self.boundaries) + 1)
        self.count = 0
        self.sum = 0.0
        self._lock = threading.Lock()

    def Observe(self, value: float):
        k = bisect.bisect_left(self.boundaries, value)
        with self._lock:
            self.counts[k] += 1
            self.count += 1
            self.sum += value


class _MapFamily(Family):
    def __init__(self, make):
        self._make = make
        self.metrics: Dict[Tuple, object] = {}
        self._lock = threading.Lock()

    def Add(self, labels: Dict[str, str]):
        key = tuple(sorted(labels.items()))
        with self._lock:
            if key not in self.metrics:
                self.metrics[key] = self._make()
            return self.metrics[key]

    def find(self, labels: Dict[str, str]):
        return self.metrics.get(tuple(sorted(labels.items())))


class InMemoryFamilyFactory(FamilyFactory):
    def __init__(self):
        self.families: Dict[str, _MapFamily] = {}

    def _make(self, name, make):
        if name not in self.families:
            self.families[name] = _MapFamily(make)
        return self.families[name]

    def NewCounterFamily(self, name, description):
        return self._make(name, ValueCounter)

    def NewGaugeFamily(self, name, description):
        return self._make(name, ValueGauge)

    def NewHistogramFamily(self, name, description, boundaries):
        return self._make(name, lambda: BucketHistogram(boundaries))

    def get(self, name, labels=None):
        """The metric of family `name` with `labels` (None if absent)."""
        f = self.families.get(name)
        return None if f is None else f.find(labels or {})


# ---- common::Histogram -------------------------------------------------------
def _g(v) -> str:
    return "%g" % float(v)


class ScoreHistogram:
    """common::Histogram (common/histogram.cc:27-75): float values, ToString in
    the reference's float32 arithmetic and absl formatting (integers in
    decimal, floats with six significant digits)."""

    def __init__(self):
        self.values: List[np.float32] = []

    def Add(self, value: float):
        self.values.append(np.float32(value))

    def __len__(self):
        return len(self.values)

    def ToString(self, buckets: int) -> str:
        if buckets < 1:
            raise ValueError("buckets must be >= 1")  # CHECK_GE
        f32 = np.float32
        vals = self.values
        if not vals:
            return "Count: 0"
        n = len(vals)
        mn, mx = min(vals), max(vals)
        acc = f32(0.0)
        for v in vals:  # std::accumulate(..., 0.f): in order, in float
            acc = f32(acc + v)
        mean = f32(acc / f32(n))
        result = f"Count: {n}  Min: {_g(mn)}  Max: {_g(mx)}  Mean: {_g(mean)}"
        if mn == mx:
            return result
        lower = mn
        total = 0
        for i in range(buckets):
            if i + 1 == buckets:
                upper = mx
            else:
                upper = f32(f32(f32(mx * f32(i + 1)) / f32(buckets)) +
                            f32(f32(mn * f32(buckets - i - 1)) / f32(buckets)))
            last = i + 1 == buckets
            count = sum(1 for v in vals if lower <= v and (v <= upper if last else v < upper))
            total += count
            result += "\n[%f, %f%s" % (float(lower), float(upper), "]" if last else ")")
            bar = (count * 20 + n // 2) // n
            result += "\t" + "".join(" " if k < 20 - bar else "#" for k in range(20))
            result += (f"\tCount: {count} ({_g(f32(f32(count * f32(100.0)) / f32(n)))}%)"
                       f"\tTotal: {total} ({_g(f32(f32(total * f32(100.0)) / f32(n)))}%)")
            lower = upper
        return result
