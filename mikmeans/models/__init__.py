"""Algorithm families: Lloyd (full batch), mini-batch, initialisation, trait-card rooms."""
from .init import floyd_sample, init_kmeanspp, init_random, resolve_init
from .lloyd import IterStats, LloydEngine
from .minibatch import MiniBatchEngine

__all__ = ["LloydEngine", "IterStats", "MiniBatchEngine", "resolve_init", "init_kmeanspp",
           "init_random", "floyd_sample"]
