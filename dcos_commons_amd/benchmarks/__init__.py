"""Benchmarks for the headline metric (deploy wall-clock + recovery MTTR)."""
