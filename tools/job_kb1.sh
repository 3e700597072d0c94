set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/h2sw; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "conv or deconv or upsample" > $O/t_conv.log 2>&1
for i in 1 2; do
  RF_LIB=$R/renderformer_amd/lib/librfhip_base.so KB_F16_ONLY=1 KB_CONV_TILES=h2 timeout -k 10 200 python -u tools/kbench.py conv > $O/kb_base$i.log 2>&1
  KB_F16_ONLY=1 KB_CONV_TILES=h2,h2db4,h2db8 timeout -k 10 200 python -u tools/kbench.py conv > $O/kb_new$i.log 2>&1
done
bash tools/gpu.sh ab h2sw "RF_LIB=$R/renderformer_amd/lib/librfhip_base.so" "RF_LIB=$R/renderformer_amd/lib/librfhip.so"
echo ok
