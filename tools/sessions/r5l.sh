#!/bin/bash
# Round 5: exact-mode time split of the per-position scalar bookkeeping (variant builds of
# tools/variants/: 6 no weight select and skip test, 7 no skip test; results wrong by construction).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/${1:-r5l}; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2; do
for v in base 6 7; do
  if [ $v = base ]; then L=""; else L="tools/variants/libniidmix_split$v.so"; fi
  NIIDMIX_LIB=$L timeout -k 10 300 python -u tools/exact_probe.py --rts 16 --metas rem8 --reps 2 --no-check > $O/exact_probe_$v.txt 2>&1 || { echo "probe $v failed"; tail -5 $O/exact_probe_$v.txt; exit 3; }
  echo "variant $v"; grep SUMMARY $O/exact_probe_$v.txt
done; done
echo done
