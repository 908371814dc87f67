# round 6 A/B: the drop-in checksum()'s per-call cost by length, before and
# after the short-buffer path (scripts/build/dropin_{old,new}, built from
# csum_cpu.c of the two commits by scripts/dropin_short_ab_build.sh)
cd $GRAFT_REPO_ROOT || exit 1
for k in 1 2 3; do
  for v in old new; do
    printf '{"build": "%s", "ns_per_call": ' $v >> gpurun_out/dropin_ab.jsonl
    timeout -k 10 60 taskset -c 2 scripts/build/dropin_$v 2000000 20 24 40 60 64 72 536 800 1500 | tr -d '\n' >> gpurun_out/dropin_ab.jsonl || exit 1
    echo "}" >> gpurun_out/dropin_ab.jsonl
  done
done
