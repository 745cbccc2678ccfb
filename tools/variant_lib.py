"""Build a variant of liblsp_hip.so for same-box A/B runs: the library's
objects with some sources recompiled under extra -D flags, linked into
abl/<name>.so (git-ignored; travels to the GPU box with gpurun).
Usage: python tools/variant_lib.py <name> <src.hip[,src2...]> [-DFLAG=V ...]
Run the in-tree build first (python -m linea_stark_prover_amd.build)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from linea_stark_prover_amd import build as B  # noqa: E402


def main():
    name, srcs, flags = sys.argv[1], sys.argv[2].split(","), sys.argv[3:]
    out_dir = os.path.join(ROOT, "abl", name)
    os.makedirs(out_dir, exist_ok=True)
    objs = []
    for s in B.SOURCES:
        obj = os.path.join(B.BUILD, os.path.splitext(s)[0] + ".o")
        if s in srcs:
            vobj = os.path.join(out_dir, os.path.splitext(s)[0] + ".o")
            cmd = [B.HIPCC] + B.CFLAGS + flags + (["-x", "hip"] if s.endswith(".cpp") else []) + \
                ["-c", os.path.join(B.CSRC, s), "-o", vobj]
            subprocess.run(cmd, check=True)
            obj = vobj
        objs.append(obj)
    lib = os.path.join(ROOT, "abl", name + ".so")
    subprocess.run([B.HIPCC, "-shared", f"--offload-arch={B.ARCH}", "-o", lib] + objs + ["-lpthread", "-ldl"],
                   check=True)
    print(lib)


if __name__ == "__main__":
    main()
