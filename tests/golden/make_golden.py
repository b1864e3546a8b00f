"""Regenerates the generated golden fixtures (see README.md).  Run from the repo root:
    python tests/golden/make_golden.py
Needs /root/reference/uniprot_arg.fasta only to (re)create uniprot_arg.fasta.gz."""
import gzip
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from common import ROOT, edges_sha256, parse_fasta_bytes  # noqa: E402

sys.path.insert(0, ROOT)
from oracle.oracle import Oracle  # noqa: E402

SURVEY_COUNTERS = {  # SURVEY.md §8c golden counters table (independent restatement)
    "5": {"distinct": 430853, "repeat": 231253, "sum_cdf2": 258621291, "sum_w_diff": 5300233,
          "n_edges": 4350628, "n_align": 465, "pairs_any": 15105756, "sum_S": 3388895},
    "7": {"distinct": 731043, "repeat": 288551, "sum_cdf2": 161007253, "sum_w_diff": 99250,
          "n_edges": 22732, "n_align": 463, "pairs_any": 9022016, "sum_S": 3371829},
}


def main():
    gz = os.path.join(HERE, "uniprot_arg.fasta.gz")
    src = "/root/reference/uniprot_arg.fasta"
    if not os.path.exists(gz):
        with open(src, "rb") as f, gzip.open(gz, "wb", compresslevel=9) as g:
            g.write(f.read())
    with gzip.open(gz, "rb") as f:
        data = f.read()
    res, off, cls, _ = parse_fasta_bytes(data)
    out = {"dataset_sha256": hashlib.sha256(data).hexdigest(), "n_proteins": len(off) - 1}
    for k in (5, 7):
        o = Oracle(res, off, cls, k=k, threads=os.cpu_count() or 1)
        p, q, w = o.pairs()
        c = o.counters()
        for key, val in SURVEY_COUNTERS[str(k)].items():
            assert c[key] == val, (k, key, c[key], val)
        out[str(k)] = dict(SURVEY_COUNTERS[str(k)], max_df=c["max_df"], n_windows=c["n_windows"],
                           edges_sha256=edges_sha256(p, q, w))
    with open(os.path.join(HERE, "uniprot_counters.json"), "w") as f:
        json.dump(out, f, indent=1)

    import uniprot_kmer_based_clustering_amd as K
    synth = {}
    for n, seed, law in ((64, 1, 0), (1000, 2, 0), (500, 5, 1)):
        path = f"/tmp/kmp_synth_{n}_{seed}_{law}.fasta"
        K.write_synth_fasta(path, n, seed, law)
        with open(path, "rb") as f:
            synth[f"{n}_{seed}_{law}"] = hashlib.sha256(f.read()).hexdigest()
        os.remove(path)
    with open(os.path.join(HERE, "synth_sha256.json"), "w") as f:
        json.dump(synth, f, indent=1)


if __name__ == "__main__":
    main()
