"""Observability (absent in the reference: SageMaker Debugger/profiler is disabled at ``launch.py:53``).

* :class:`ThroughputMeter` — whole-node sequences/sec from device events, ``metrics.jsonl`` and a
  final ``benchmark.json`` (SURVEY.md §5 'Metrics / logging / observability').
* :class:`ProfilerCallback` / :func:`range` — roctx ranges around the step phases and a
  ``torch.profiler`` window exported as a Chrome trace (rocprofv3 recipes: ``bench/rocprof_recipes.md``).
"""
from .profiler import ProfilerCallback, range, ranges_enabled, set_ranges
from .throughput import ThroughputMeter

__all__ = ["ThroughputMeter", "ProfilerCallback", "range", "ranges_enabled", "set_ranges"]
