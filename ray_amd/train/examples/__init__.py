"""Runnable Ray Train workloads (reference: release/air_tests/air_benchmarks/workloads)."""
