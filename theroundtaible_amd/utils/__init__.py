"""Host utilities: atomic IO, timing/metrics, tracing, logging."""
