# lab_clocks.py: power and clocks under load, per workload and kernel (and the
# plain read probe over the same buffer), one process each.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/clk
export TMPDIR=/tmp
i=0
for spec in ${CLK_SPECS:-mixed:auto tcp1500:auto mixed:probe tcp1500:probe mixed:auto}; do
  i=$((i+1)); wl=${spec%%:*}; mode=${spec##*:}
  CLK_WORKLOAD=$wl CLK_MODE=$mode timeout -k 10 150 python scripts/lab_clocks.py gpurun_out/clk/q$i.json 3 > gpurun_out/clk/q$i.log 2>&1
  rc=$?; grep window gpurun_out/clk/q$i.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/clk/q$i.log; exit $rc; }
done
exit 0
