source scripts/gpu_step.sh
PREV=$(pwd)/ablib/libsimplex_prev.so
for v in new prev; do
  if [ $v = prev ]; then export SIMPLEX_LIB_PATH=$PREV; else unset SIMPLEX_LIB_PATH; fi
  step ss_$v 300 python -u tools/stage_stamps.py config5,config3 || exit $?
  echo "-- $v"; grep -h "stage" $O/ss_$v.log
done
