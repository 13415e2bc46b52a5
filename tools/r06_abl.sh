set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06abl; mkdir -p $O
L=channelestimationtransformer_amd
timeout -k 10 60 tools/probe/dma_probe > $O/dma_probe.txt 2>&1; echo "dma probe rc $?"; cat $O/dma_probe.txt
CET_LIB=$(pwd)/$L/libcet_feed.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/feed_tests.log 2>&1; echo "feed tests rc $?"; tail -5 $O/feed_tests.log
bash tools/ab_bench.sh $L/libcet.so $L/libcet_feed.so $L/libcet_abl_WL1.so $L/libcet_abl_PL1.so $L/libcet_abl_LN.so $L/libcet_abl_DEC.so 2>&1 | tee $O/ab.log
bash tools/stamps_ab.sh $O/stamps $L/libcet_c2st.so $L/libcet_c2st_feed.so $L/libcet_c2st_wl1.so
