"""Cross-cutting helpers: roctx tracing (trace)."""
from .trace import profiler_start, profiler_stop, range_ctx  # noqa: F401
