"""Runtime utilities: roctx tracing ranges and phase timers, NaN/Inf guards, JSONL
metrics, and a step watchdog (SURVEY.md sections 5.1-5.5)."""
from .guards import nonfinite, check_finite
from .jsonl import JsonlLogger
from .tracing import PhaseTimer, mark, trace_range
from .watchdog import StepWatchdog

__all__ = ["nonfinite", "check_finite", "JsonlLogger", "PhaseTimer", "mark", "trace_range",
           "StepWatchdog"]
