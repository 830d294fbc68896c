set -o pipefail
mkdir -p gpurun_out/discovery
cd gpurun_out/discovery
(timeout -k 5 60 amd-smi static --json > amd_smi_static.json 2> amd_smi_static.err; echo "rc=$?" >> amd_smi_static.err)
(timeout -k 5 60 amd-smi list --json > amd_smi_list.json 2> amd_smi_list.err; echo "rc=$?" >> amd_smi_list.err)
(timeout -k 5 60 amd-smi topology --json > amd_smi_topology.json 2> amd_smi_topology.err; echo "rc=$?" >> amd_smi_topology.err)
(timeout -k 5 60 amd-smi xgmi --json > amd_smi_xgmi.json 2> amd_smi_xgmi.err; echo "rc=$?" >> amd_smi_xgmi.err)
(timeout -k 5 60 rocminfo > rocminfo.txt 2> rocminfo.err; echo "rc=$?" >> rocminfo.err)
(timeout -k 5 60 rocm-smi --showtopo --json > rocm_smi_topo.json 2> rocm_smi_topo.err; echo "rc=$?" >> rocm_smi_topo.err)
mkdir -p kfd
if [ -d /sys/class/kfd/kfd/topology ]; then
  cp /sys/class/kfd/kfd/topology/generation_id kfd/ 2>/dev/null || true
  cp /sys/class/kfd/kfd/topology/system_properties kfd/ 2>/dev/null || true
  for n in /sys/class/kfd/kfd/topology/nodes/*; do
    b=$(basename $n); mkdir -p kfd/nodes/$b
    cp $n/properties kfd/nodes/$b/ 2>/dev/null || true
    cp $n/name kfd/nodes/$b/ 2>/dev/null || true
    cp $n/gpu_id kfd/nodes/$b/ 2>/dev/null || true
    for l in $n/io_links/* $n/p2p_links/*; do
      [ -e "$l/properties" ] || continue
      d=kfd/nodes/$b/$(basename $(dirname $l))/$(basename $l); mkdir -p $d; cp $l/properties $d/ 2>/dev/null || true
    done
  done
fi
ls -R kfd | head -50 > kfd_listing.txt
echo HIP_VISIBLE_DEVICES=$HIP_VISIBLE_DEVICES ROCR_VISIBLE_DEVICES=$ROCR_VISIBLE_DEVICES > env.txt
nproc >> env.txt
echo done
