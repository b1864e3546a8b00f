"""Pipelined submissions on config 3 with stage timing: per-step stage times (diagnostic)."""
import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import uniprot_kmer_based_clustering_amd as K
from uniprot_kmer_based_clustering_amd.device import DevicePipeline
b = K.synth(100000, 3)
pipe = DevicePipeline(b, 7, "cuda:0")
pipe.set_stage_timing(True)
prev = None
for i in range(12):
    t = pipe.submit()
    if prev is not None:
        pipe.wait(prev)
        print(i, pipe.graph_replays(), [round(x, 4) for x in pipe.postings_stats.stage_ms[:6]], flush=True)
    prev = t
pipe.wait(prev)
print('last', [round(x, 4) for x in pipe.postings_stats.stage_ms[:6]])
