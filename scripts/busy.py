"""Busy fraction of the GPU from a rocprofv3 kernel trace: the union of kernel [start, end) intervals
over windows of the run, so gaps where no kernel runs on any stream show up.  Prints the whole trace's
span and busy time, and the same over the last 80 % of the span (past setup and the latency pass)."""
import csv
import sys


def main(path):
    iv, names = [], []
    for r in csv.DictReader(open(path)):
        iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "")[:60]))
    iv.sort()
    names = [n for _, _, n in iv]
    iv = [(s, e) for s, e, _ in iv]
    t0, t1 = iv[0][0], max(e for _, e in iv)

    def busy(lo, hi):
        tot, cur_s, cur_e = 0, None, None
        for s, e in iv:
            s, e = max(s, lo), min(e, hi)
            if e <= s:
                continue
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    tot += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            tot += cur_e - cur_s
        return tot

    span = t1 - t0
    print(f"kernels {len(iv)}, span {span / 1e9:.3f} s, busy {busy(t0, t1) / 1e9:.3f} s ({busy(t0, t1) / span:.3f})")
    for frac in (0.5, 0.2):
        lo = t1 - int(span * frac)
        b = busy(lo, t1)
        print(f"last {frac:.0%} of the span: busy {b / 1e9:.3f} of {(t1 - lo) / 1e9:.3f} s ({b / (t1 - lo):.3f})")
    # idle gaps over the last half: size histogram and the kernels on either side of the largest
    lo = t1 - span // 2
    gaps, cur_e, prev = [], None, None
    for (s, e), n in zip(iv, names):
        if e <= lo:
            continue
        if cur_e is not None and s > cur_e:
            gaps.append((s - cur_e, prev, n))
        if cur_e is None or e > cur_e:
            cur_e, prev = e, n
    bins = [1e3, 1e4, 5e4, 1e5, 1e6, 1e9]
    tot = sum(g for g, _, _ in gaps)
    print(f"gaps in the last half: {len(gaps)}, {tot / 1e9:.3f} s")
    lo_b = 0
    for b in bins:
        sel = [g for g, _, _ in gaps if lo_b <= g < b]
        print(f"  {lo_b / 1e3:>8.0f}-{b / 1e3:<8.0f} us: {len(sel):7d} gaps, {sum(sel) / 1e9:.3f} s")
        lo_b = b
    pairs = {}
    for g, a, b in gaps:
        k = (a, b)
        c, t = pairs.get(k, (0, 0))
        pairs[k] = (c + 1, t + g)
    print("kernel pairs around gaps, by total gap time:")
    for (a, b), (c, t) in sorted(pairs.items(), key=lambda x: -x[1][1])[:15]:
        print(f"  {t / 1e6:8.1f} ms {c:6d}x  {a} -> {b}")


if __name__ == "__main__":
    main(sys.argv[1])
