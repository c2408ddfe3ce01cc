"""Build an alternative libwsmc.so with extra preprocessor definitions, for A/B runs on one box
(select it with WSMC_LIB=<path>): python tools/build_variant.py <name> -DFOO=0 ...
Output: tools/variants/<name>/libwsmc.so (git-ignored, travels with the tree)."""
import pathlib
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "weightedsampling.jl_amd"))
import build as B  # noqa: E402

name, defs = sys.argv[1], sys.argv[2:]
out = ROOT / "tools" / "variants" / name
out.mkdir(parents=True, exist_ok=True)
B.write_jit_headers()
cc = B.hipcc()


def one(src):
    obj = out / (pathlib.Path(src).stem + ".o")
    r = subprocess.run([cc, *B.COMMON, *defs, "-I", str(B.OBJDIR), "-c", str(B.CSRC / src), "-o", str(obj)],
                       capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(r.stderr)
    return obj


with ThreadPoolExecutor(max_workers=len(B.SOURCES)) as ex:
    objs = list(ex.map(one, B.SOURCES))
lib = out / "libwsmc.so"
r = subprocess.run([cc, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(lib),
                    "-L/opt/rocm/lib", "-lrccl", "-lhiprtc", "-Wl,-rpath,/opt/rocm/lib"], capture_output=True, text=True)
if r.returncode:
    raise SystemExit(r.stderr)
for o in objs:
    o.unlink()
print(lib)
