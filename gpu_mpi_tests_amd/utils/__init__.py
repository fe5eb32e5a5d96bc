"""Cross-cutting helpers: roctx tracing (trace), timers/statistics (timer), JSON reports (report)."""
from .report import json_line, write_jsonl  # noqa: F401
from .timer import Stats, Timer  # noqa: F401
from .trace import profiler_start, profiler_stop, range_ctx  # noqa: F401
