"""GPU busy fraction per eager step from a rocprofv3 --kernel-trace CSV (one step = the kernels between two
launches of the step's last kernel, e.g. the optimiser's multi_tensor_apply): the union of kernel intervals over
the step's wall span, and the per-step kernel time by name. Says whether an eager caller loop (C5) is
device- or host-bound. python tools/kernel_trace_busy.py TRACE.csv [STEP_KERNEL_SUBSTRING] [KERNELS_PER_STEP]"""
import collections
import csv
import sys


def main(path, marker="multi_tensor_apply", per_step=None):
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    ends = [e for s, e, n in ks if marker in n]
    steps = []
    for a, b in zip(ends[:-1], ends[1:]):
        iv = [(s, e, n) for s, e, n in ks if s >= a and e <= b]
        if len(iv) < 8 or (per_step and len(iv) != int(per_step)):
            continue
        busy, cs, ce = 0, None, None
        for s, e, _ in iv:
            if ce is None or s > ce:
                if ce is not None:
                    busy += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        steps.append((b - a, busy, iv))
    if not steps:
        raise SystemExit("no steps found")
    steps = steps[1:]  # the first counted step follows the warm-up
    span = sorted(s[0] for s in steps)[len(steps) // 2] / 1e3
    busy = sorted(s[1] for s in steps)[len(steps) // 2] / 1e3
    print(f"steps {len(steps)}, kernels per step {len(steps[0][2])}: median wall {span:.1f} us (profiled), "
          f"GPU busy {busy:.1f} us = {busy / span:.3f}")
    agg = collections.defaultdict(lambda: [0, 0.0])
    for _, _, iv in steps:
        for s, e, n in iv:
            k = n.split("(")[0][:80]
            agg[k][0] += 1
            agg[k][1] += e - s
    ns = len(steps)
    for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"  {c / ns:5.1f} x {t / c / 1e3:6.2f} us = {t / ns / 1e3:7.1f} us/step  {k}")


if __name__ == "__main__":
    main(*sys.argv[1:])
