"""Utilities: timers, profiling markers, rocprofv3 summary parsing."""
