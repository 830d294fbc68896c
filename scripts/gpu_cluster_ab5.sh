# Same-box interleaved cluster-mode A/B (round 5): ab_trees/head (before the helper-side sandbox
# set-up) vs this tree, and this tree with a 0.5 ms switch interval in the cluster process (master +
# agents). 8 and 1 pods, 6 cycles per run, 4 rounds, order rotating.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cab5
root=$(pwd)
run() {  # label tree n extra...
  local label=$1 tree=$2 n=$3; shift 3
  (cd "$tree" && timeout -k 10 240 python -u -m dcos_commons_amd.benchmarks.cluster_bench --agents $n --cycles 6 "$@" \
    | sed "s|^|$label n$n |" >> "$root/gpurun_out/cab5/res.txt" 2>> "$root/gpurun_out/cab5/err.txt")
}
for i in 1 2 3 4; do
  for n in 8 1; do
    case $((i % 3)) in
      1) run head ab_trees/head $n && run new . $n && run si05 . $n --cluster-switch-interval-ms 0.5 || exit $? ;;
      2) run new . $n && run si05 . $n --cluster-switch-interval-ms 0.5 && run head ab_trees/head $n || exit $? ;;
      0) run si05 . $n --cluster-switch-interval-ms 0.5 && run head ab_trees/head $n && run new . $n || exit $? ;;
    esac
  done
done
