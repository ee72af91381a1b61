#!/usr/bin/env python3
"""Gate-release latency of bench.py's gated window, from a rocprofv3 kernel trace of the same run.

    python tools/gate_latency.py <bench line .json> <rocprofv3 *_kernel_trace.csv>

bench.py records the host clocks of its flag store (`gate.release_clock_ns`, CLOCK_BOOTTIME and
CLOCK_MONOTONIC).  rocprofv3 stamps kernels on one of those axes; the script takes the k_stream_gate
dispatch whose end is the first after the store on either axis (the one giving a gap under 1 ms)
and prints: store -> gate wave exit, gate exit -> first rollout kernel start (the start event sits
between them), and the timed launches' span.  Output: one JSON object."""
import csv
import json
import sys


def main():
    line = json.load(open(sys.argv[1]))
    rel = line["gate"]["release_clock_ns"]
    rows = list(csv.DictReader(open(sys.argv[2])))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                 for r in rows), key=lambda k: k[0])
    best = None
    for axis, t in rel.items():
        gates = [k for k in ks if "k_stream_gate" in k[2] and k[1] >= t]
        if gates and gates[0][1] - t < 1_000_000:
            best = (axis, t, gates[0])
            break
    if best is None:
        print(json.dumps({"error": "no gate dispatch ends within 1 ms after the store on either "
                                   "clock axis"}))
        return 1
    axis, t, g = best
    after = [k for k in ks if k[0] >= g[1] and "k_rollout" in k[2]]
    n = line["config"]["timed_launches"]
    n = n["count"] if isinstance(n, dict) else len(n)
    timed = after[:n]
    out = {"clock_axis": axis,
           "store_to_gate_exit_us": (g[1] - t) / 1e3,
           "gate_wave_us": (g[1] - g[0]) / 1e3,
           "gate_exit_to_first_launch_us": (timed[0][0] - g[1]) / 1e3 if timed else None,
           "store_to_first_launch_us": (timed[0][0] - t) / 1e3 if timed else None,
           "timed_launches_span_us": (timed[-1][1] - timed[0][0]) / 1e3 if timed else None,
           "timed_kernels": [k[2][:60] for k in timed],
           "line_fixed_overhead_us": line["fixed_overhead_ms"] * 1e3,
           "line_kernel_span_us": line["roofline"]["kernel_ms_timed"] * 1e3}
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
