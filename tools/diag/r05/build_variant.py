"""Round 5: build a variant of _dlgm_hip.so in which ONE kernel source is compiled with extra hipcc flags (e.g. an
LLVM AMDGPU scheduling strategy), for same-process A/B through DLGM_HIP_LIB (tools/ab_kernels.sh).

    python tools/diag/r05/build_variant.py <tag> <source stem> <flag> [<flag> ...]
    -> build/variants/_dlgm_hip_<tag>.so  (the other objects are the in-tree build's; the in-tree library is
       (re)built from the current sources first, so it always matches them)
Prints the kernel resource usage of the variant object (VGPRs / spills) for the kernels in that source."""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[3]
sys.path.insert(0, str(ROOT / "tools"))
import build_native as bn  # noqa: E402


def main() -> int:
    tag, stem, extra = sys.argv[1], sys.argv[2], sys.argv[3:]
    bn.build()  # the in-tree objects at their current stamp
    tlib, tinc, abi = bn._torch_paths()
    import sysconfig
    common = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={bn.ARCH}", f"-I{bn.CSRC / 'include'}",
              "-Wno-unused-result", "-Wno-deprecated-declarations"]
    flags = [*common, *(f"-I{p}" for p in tinc), f"-I{sysconfig.get_paths()['include']}",
             f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1", "-DTORCH_API_INCLUDE_EXTENSION_H"]
    import hashlib
    stamp = bn._headers_stamp() + hashlib.sha1(" ".join(flags).encode()).hexdigest()[:8]
    srcs = sorted((bn.CSRC / "kernels").glob("*.hip")) + [bn.CSRC / "bindings.cpp"]
    out_dir = ROOT / "build" / "variants"
    out_dir.mkdir(parents=True, exist_ok=True)
    objs = []
    for s in srcs:
        if s.stem == stem:
            o = out_dir / f"{s.stem}.{tag}.o"
            cmd = [bn.HIPCC, *flags, *extra, "-Rpass-analysis=kernel-resource-usage", "-c", str(s), "-o", str(o)]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                print(r.stderr[-3000:])
                return 1
            for line in r.stderr.splitlines():
                if "Function Name" in line or "VGPRs:" in line or "Spill" in line or "Occupancy" in line:
                    print(line.split("remark: ")[-1])
            objs.append(o)
        else:
            objs.append(bn.BUILD / f"{s.stem}.{s.suffix[1:]}.{stamp}.o")
    kern_ld = [f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip", "-ltorch", "-lhipblaslt",
               f"-Wl,-rpath,{tlib}"]
    so = out_dir / f"_dlgm_hip_{tag}.so"
    r = subprocess.run([bn.HIPCC, "-shared", "-fPIC", f"--offload-arch={bn.ARCH}", *map(str, objs), "-o", str(so),
                        *kern_ld], capture_output=True, text=True)
    if r.returncode != 0:
        print(r.stderr[-3000:])
        return 1
    print("built", so.relative_to(ROOT))
    return 0


if __name__ == "__main__":
    sys.exit(main())
