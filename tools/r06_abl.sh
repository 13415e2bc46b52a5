set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06abl; mkdir -p $O
timeout -k 10 60 tools/probe/dma_probe > $O/dma_probe.txt 2>&1; echo "dma probe rc $?"; cat $O/dma_probe.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_poison.py tests/test_gpu_layerwise.py::test_fused_layerwise_bf16_deep_k_vs_oracle tests/test_gpu_informer.py::test_encoder_split_e43_rows_with_dff128_vs_oracle -v --timeout 120 --timeout-method thread > $O/new_tests.log 2>&1; echo "new tests rc $?"; tail -5 $O/new_tests.log
L=channelestimationtransformer_amd
bash tools/ab_bench.sh $L/libcet.so $L/libcet_abl_WL1.so $L/libcet_abl_PL1.so $L/libcet_abl_LN.so $L/libcet_abl_DEC.so 2>&1 | tee $O/ab.log
bash tools/stamps_ab.sh $O/stamps $L/libcet_c2st.so $L/libcet_c2st_wl1.so
