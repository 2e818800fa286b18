"""Busy fraction of the GPU from a rocprofv3 kernel trace: the union of kernel [start, end) intervals
over windows of the run, so gaps where no kernel runs on any stream show up.  Prints the whole trace's
span and busy time, and the same over the last 80 % of the span (past setup and the latency pass)."""
import csv
import sys


def main(path):
    iv = []
    for r in csv.DictReader(open(path)):
        iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    iv.sort()
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


if __name__ == "__main__":
    main(sys.argv[1])
