"""Per-rank compute of the fixed-capacity multi-GPU flow, emulated on one GPU: every rank's send
buffers are computed in turn, rank 0's receive buffers are assembled from them (exactly what the
all-to-alls would deliver), and rank 0's three stages are timed with HIP events.  Exchanges are
not included.  Diagnostic tool: python tools/time_dist_rank.py [N]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import uniprot_kmer_based_clustering_amd as K  # noqa: E402
from uniprot_kmer_based_clustering_amd.device import DevicePipeline  # noqa: E402
from uniprot_kmer_based_clustering_amd.dist import DeviceRouteStages, protein_slices  # noqa: E402


def timed(fn, reps=5):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(reps):
        out = fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps, out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    b = K.synth(n, 3)
    pipe = DevicePipeline(b, 7, "cuda:0")
    for world in (1, 2, 4, 8):
        st = DeviceRouteStages(pipe)
        sl = protein_slices(pipe.offsets_host, world)
        for attempt in range(4):
            st.begin(world)
            sends = [st.keys_route(lo, hi, world).clone() for lo, hi in sl]
            ck = st.cap_keys
            recvs = [torch.cat([s[r * ck:(r + 1) * ck] for s in sends]) for r in range(world)]
            sends2 = [st.pairs_route(recvs[r], r, world).clone() for r in range(world)]
            cp = st.cap_pairs
            recv2 = torch.cat([s[0:cp] for s in sends2])
            e, cnt = st.edges_route(recv2, 0, world)
            flags = st.flags.cpu().numpy()
            if flags[0] or flags[3]:
                st.grow(flags)
                continue
            break
        lo, hi = sl[0]
        t1, _ = timed(lambda: st.keys_route(lo, hi, world))
        t2, _ = timed(lambda: st.pairs_route(recvs[0], 0, world))
        t3, _ = timed(lambda: st.edges_route(recv2, 0, world))
        print(f"world={world} rank0: keys_route {t1:.3f} ms  pairs_route {t2:.3f} ms  edges_route {t3:.3f} ms  "
              f"total {t1 + t2 + t3:.3f} ms | exchange bytes/rank: keys {world * ck * 8 / 1e6:.1f} MB, "
              f"pairs {world * cp * 8 / 1e6:.1f} MB | edges rank0 {int(cnt.item())}")


if __name__ == "__main__":
    main()
