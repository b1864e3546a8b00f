"""Config 1 (uniprot_arg.fasta, k = 5: the split step) with graphs on and off: ms per step and the
graph replays (diagnostic for the split step's front graph)."""
import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import bench
from uniprot_kmer_based_clustering_amd.device import DevicePipeline
b = bench.load_batch("config1")
pipe = DevicePipeline(b, 5, "cuda:0")
for graphs in (True, False, True):
    pipe.set_graph(graphs)
    for _ in range(4):
        pipe.step()
    torch.cuda.synchronize()
    r0 = pipe.graph_replays()
    t0 = time.perf_counter()
    for _ in range(20):
        pipe.step()
    torch.cuda.synchronize()
    print("graphs", graphs, "ms/step", round((time.perf_counter() - t0) / 20 * 1e3, 4), "replays", pipe.graph_replays() - r0,
          "heavy", pipe.last_heavy(), flush=True)
