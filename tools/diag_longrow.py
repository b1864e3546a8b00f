"""Diagnostic: layout/tail decisions on the long-row p-shard test input."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import uniprot_kmer_based_clustering_amd as K  # noqa: E402
from uniprot_kmer_based_clustering_amd.device import DevicePipeline  # noqa: E402
from common import make_batch  # noqa: E402

rng = np.random.default_rng(5)
alpha = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", dtype=np.uint8)
rnd = lambda m: alpha[rng.integers(0, 20, m)].tobytes()  # noqa: E731
base = rnd(700)
seqs = [base] + [rnd(40) + base[i:i + 7] + rnd(40) for i in range(650)]
res, off, cls = make_batch(seqs, ["a"] + ["b"] * 650)
pipe = DevicePipeline(K.Proteins(res, off, cls), 7, "cuda:0")
for _ in range(2):
    m = pipe.step(engine="residues")
    torch.cuda.synchronize()
    print("edges", m, pipe.last_layout(), pipe.last_tail(), pipe.postings_stats.as_dict())
