"""Utilities: metrics, trait analytics, JS-exact JSON, checkpoints, profiling."""
from . import checkpoint, jsjson, metrics, profiling, traits

__all__ = ["checkpoint", "jsjson", "metrics", "profiling", "traits"]
