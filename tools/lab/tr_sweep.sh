bash tools/lab/run_trace.sh "-DNO_TRACE" "32 9" || exit 1
bash tools/lab/run_trace.sh "-DNO_TRACE -DLK_WEIGHT_AUX=0" "32 9" || exit 1
