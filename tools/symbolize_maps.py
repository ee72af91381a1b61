"""Map the unsymbolized PCs of a glog stack trace (the rocprofv3 exit-time SIGSEGV records) to
library + offset with the process's /proc/self/maps (tools/coop_exit_probe.py), then to a symbol
with llvm-symbolizer (same image here as on the GPU box: the libraries are the same files).

    python tools/symbolize_maps.py ERR_FILE MAPS_FILE"""
import re
import subprocess
import sys

SYM = "/opt/rocm/lib/llvm/bin/llvm-symbolizer"


def load_maps(path):
    out = []
    for line in open(path):
        p = line.split()
        if len(p) < 6:
            continue
        lo, hi = (int(x, 16) for x in p[0].split("-"))
        out.append((lo, hi, int(p[2], 16), p[5]))
    return out


def base_of(maps, path):
    return min(lo - off for lo, hi, off, p in maps if p == path)


def main():
    err, maps_path = sys.argv[1], sys.argv[2]
    maps = load_maps(maps_path)
    pcs = [int(m.group(1), 16) for m in re.finditer(r"@\s+0x([0-9a-f]+)", open(err).read())]
    for pc in pcs:
        hit = next(((lo, hi, off, p) for lo, hi, off, p in maps if lo <= pc < hi), None)
        if hit is None:
            print(f"0x{pc:x}  (not mapped at exit)")
            continue
        lo, hi, off, path = hit
        rel = pc - base_of(maps, path)
        sym = ""
        try:
            sym = subprocess.run([SYM, "--obj", path, "-f", "-C", hex(rel)], capture_output=True,
                                 text=True, timeout=30).stdout.strip().splitlines()[0]
        except Exception as ex:  # noqa: BLE001
            sym = f"({type(ex).__name__})"
        print(f"0x{pc:x}  {path}+0x{rel:x}  {sym}")


if __name__ == "__main__":
    main()
