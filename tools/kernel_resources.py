"""Per-kernel register / scratch usage of the built libwxalign.so (development tool):
unbundles the gfx950 code object and prints the metadata notes of the matching kernels."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def notes(so):
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "k.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", so], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        txt = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    # the metadata keys of a kernel are sorted: those before ".name" (group_segment_fixed_size)
    # belong to the kernel whose name follows
    out, cur, pending = [], {}, {}
    for line in txt.splitlines():
        m = re.match(r"\s+\.(name|vgpr_count|sgpr_count|private_segment_fixed_size|group_segment_fixed_size|vgpr_spill_count):\s+(\S+)", line)
        if m:
            k, v = m.groups()
            if k == "name":
                cur = {"name": v, **pending}
                pending = {}
                out.append(cur)
            elif k < "name":
                pending[k] = v
            else:
                cur[k] = v
    names = subprocess.run(["c++filt"], input="\n".join(o["name"] for o in out), capture_output=True,
                           text=True).stdout.splitlines()
    for o, n in zip(out, names):
        o["name"] = n
    return out


if __name__ == "__main__":
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "whisperx_amd", "libwxalign.so")
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else "align_dp")
    # a sharded build links several code objects; the unbundler reads only the first, so read
    # the build's objects (build/obj/<lib>/*.o) when they are there
    import glob
    objs = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "..", "build", "obj",
                                         os.path.basename(so).replace(".so", ""), "*.o")))
    for o in [x for f in (objs or [so]) for x in notes(f)]:
        if pat.search(o["name"]):
            print(f"{o['name'][:60]:60s} vgpr {o.get('vgpr_count'):>4} sgpr {o.get('sgpr_count'):>4} "
                  f"scratch {o.get('private_segment_fixed_size'):>5} lds {o.get('group_segment_fixed_size'):>6} "
                  f"spill {o.get('vgpr_spill_count')}")
