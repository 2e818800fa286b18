# Full kernel trace of boot_test (logn 14, 2 bootstraps) -> gpurun_out/boot_trace (per-launch CSV)
set -u
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/boot_trace
timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/boot_trace" -o boot --output-format csv -- "$R/build/boot_test" 14 ${REPS:-2} > gpurun_out/boot_trace/boot.log 2>&1
rc=$?
f=$(find gpurun_out/boot_trace -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys, gzip
rows = list(csv.DictReader(open(sys.argv[1])))
keep = ["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z", "Workgroup_Size_X"]
with gzip.open("gpurun_out/boot_trace/trace.csv.gz", "wt") as g:
    w = csv.writer(g)
    w.writerow(keep)
    for r in rows:
        w.writerow([r.get(k, "") for k in keep])
print(len(rows), "rows")
PY
find gpurun_out/boot_trace -name "*kernel_trace.csv" -delete
exit $rc
