"""how many host threads does the GPU box's lease actually give the CPU baseline?
The bit-exact C port (oracle/fenv_oracle.c) on 65,536 x 5 formations, ~4 s per thread count, one
formation shard per thread (bench._cpu_oracle_rate), plus what the box reports: os.cpu_count(),
the affinity mask and the cgroup CPU quota."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def cgroup_quota():
    for p in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            return p, open(p).read().strip()
        except OSError:
            pass
    return None, None


out = {"cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
       "cgroup": cgroup_quota(), "rates": {}}
for t in [int(x) for x in (sys.argv[1:] or ["1", "8", "16", "24", "32", "64"])]:
    r, k, el = bench._cpu_oracle_rate(65536, 5, 8, t, 4.0)
    out["rates"][t] = {"agent_steps_per_s": r, "min_steps_per_shard": k, "seconds": el}
    print(t, f"{r:.3e}", flush=True)
print(json.dumps(out))
