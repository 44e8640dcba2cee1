"""Parity margins of a GPU test log run with -s (every tests/helpers.report line, '[parity] ...'): per line the
checked quantity, entries, worst err/limit, the ill-conditioned entries (judged by the oracle's float64
shadow, held to the bar + 10x the f32 oracle's own error) and the vs-f64 ratios (GPU / f32 oracle, in units
of the bar); then the worst line per test. python tools/parity_summary.py LOG > SUMMARY"""
import re
import sys

PAT = re.compile(r"\[parity\] (?P<name>.*?): n = (?P<n>\d+), max\|err\| = (?P<err>\S+), scale = (?P<scale>\S+), "
                 r"worst err/limit = (?P<wl>[^, ]+)(?:, ill-conditioned = (?P<ill>\d+))?(?:, vs f64: GPU (?P<g64>\S+) / "
                 r"f32 oracle (?P<o64>\S+) of the bar)? at")


def main(path):
    test = None
    rows = []
    for line in open(path, errors="replace"):
        m = re.match(r"(tests/\S+::\S+)", line)
        if m:
            test = m.group(1).split("::")[1]
        for p in PAT.finditer(line):
            rows.append((test, p.group("name"), int(p.group("n")), float(p.group("wl")),
                         int(p.group("ill")) if p.group("ill") else None,
                         p.group("g64"), p.group("o64")))
    print(f"{len(rows)} [parity] lines from {path}")
    print("columns: worst err/limit; ill-conditioned entries; max distance to the float64 shadow in units of the bar, "
          "of the GPU and of the f32 oracle, and their ratio (> 1: the GPU is farther from f64 than the f32 oracle)")
    print(f"{'test':58s} {'quantity':52s} {'n':>8s} {'err/lim':>8s} {'ill':>6s} {'GPU/f64':>9s} {'f32orc/f64':>10s} "
          f"{'ratio':>6s}")
    farther = []
    for t, nm, n, wl, ill, g, o in rows:
        ratio = ""
        if g is not None and o is not None:
            gf, of = float(g), float(o)
            ratio = f"{gf / of:.2f}" if of > 0 else ""
            if gf > of and gf > 1.0:
                farther.append((t, nm, gf, of))
        print(f"{(t or '?')[:58]:58s} {nm[:52]:52s} {n:8d} {wl:8.3f} {'' if ill is None else ill:>6} "
              f"{g or '':>9s} {o or '':>10s} {ratio:>6s}")
    worst = max(rows, key=lambda r: r[3]) if rows else None
    if worst:
        print(f"\nworst err/limit over all lines: {worst[3]:.3f} ({worst[0]}: {worst[1]})")
    print(f"\nquantities where the GPU is farther from the float64 shadow than the f32 oracle (and more than one "
          f"bar): {len(farther)}")
    for t, nm, gf, of in sorted(farther, key=lambda r: -r[2] / r[3]):
        print(f"  {(t or '?')[:58]:58s} {nm[:52]:52s} GPU {gf:9.3f}  f32 oracle {of:9.3f}  ratio {gf / of:.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
