"""Test-side alias of the synthetic generators (pacmann_amd/synth.py)."""
from pacmann_amd.synth import *  # noqa: F401,F403
from pacmann_amd.synth import clustered_vectors, knn_graph, msmarco_like_vectors, random_graph, sift_like_vectors  # noqa: F401
