#!/usr/bin/env bash
# Stage the reference's UNCHANGED framework packages (svc.yml + config templates + universe/) into
# the gitignored ref_inputs/ so a GPU-box run (which gets only this tree) can benchmark them.
# Never committed; remove with `rm -rf ref_inputs` after the run.
set -euo pipefail
REF=${SDK_REFERENCE_ROOT:-/root/reference}
cd "$(dirname "$0")/.."
rm -rf ref_inputs
for fw in cassandra hdfs helloworld; do
  mkdir -p "ref_inputs/frameworks/$fw/src/main"
  cp -r "$REF/frameworks/$fw/src/main/dist" "ref_inputs/frameworks/$fw/src/main/dist"
  cp -r "$REF/frameworks/$fw/universe" "ref_inputs/frameworks/$fw/universe"
done
echo "staged $(find ref_inputs -type f | wc -l) files under ref_inputs/"
