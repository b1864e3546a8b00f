"""Per-kernel resources of a device object (VGPRs, SGPRs, spills, LDS): compiles a .hip with
--cuda-device-only and parses llvm-readelf --notes.  Usage: kernel_resources.py file.hip [-I dir] [-D macro] [filter]"""
import re
import subprocess
import sys
import tempfile

src = sys.argv[1]
inc = [a for a in sys.argv[2:] if a.startswith("-I")] or ["-I/root/repo/include"]
inc += [a for a in sys.argv[2:] if a.startswith("-D")]
flt = [a for a in sys.argv[2:] if not a.startswith(("-I", "-D"))]
with tempfile.TemporaryDirectory() as d:
    o = f"{d}/k.o"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", *inc,
                    "-I/root/repo/uniprot_kmer_based_clustering_amd/csrc", "--cuda-device-only",
                    "--no-gpu-bundle-output", "-c", src, "-o", o], check=True)
    notes = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", o], capture_output=True,
                           text=True).stdout
blocks = notes.split("  - .agpr_count:")[1:]
for b in blocks:
    def f(key):
        m = re.search(r"\." + key + r":\s+(\S+)", b)
        return m.group(1) if m else "?"
    name = f("name")
    if flt and not any(x in name for x in flt):
        continue
    print(f"{name[:90]:90s} vgpr {f('vgpr_count'):>4} sgpr {f('sgpr_count'):>4} vspill {f('vgpr_spill_count'):>3} "
          f"sspill {f('sgpr_spill_count'):>3} lds {f('group_segment_fixed_size'):>6} priv {f('private_segment_fixed_size')}")
