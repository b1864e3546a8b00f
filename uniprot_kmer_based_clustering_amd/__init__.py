"""MI355X-native k-mer pair engine for the hot path of Isabella136/uniprot_kmer_based_clustering.

libkmerpair.so (hand-written HIP for gfx950 behind the C ABI of include/kmerpair.h) does
the work; this package is the Python face used by tests, bench.py and the multi-GPU driver.
"""
from . import _lib  # noqa: F401
from .engine import (Edges, EdgeSet, KmerPairEngine, Mphf, Proteins, digest_term, read_fasta, synth,  # noqa: F401
                     write_synth_fasta)

__all__ = ["KmerPairEngine", "EdgeSet", "Mphf", "Proteins", "Edges", "digest_term", "read_fasta", "synth",
           "write_synth_fasta"]
