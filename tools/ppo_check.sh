set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 100 python -u tools/ppo_grad_debug.py > gpurun_out/grad_dbg.log 2>&1 || { echo "grad debug rc=$?"; tail -5 gpurun_out/grad_dbg.log; exit 1; }
grep "rel err" gpurun_out/grad_dbg.log | awk '{print $1, $5}' | tr '\n' ' '; echo
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_rollout.py tests/test_gpu_training.py > gpurun_out/pt_ppo.log 2>&1
rc=$?; tail -3 gpurun_out/pt_ppo.log; [ $rc -eq 0 ] || exit $rc
FENV_LIB_OVERRIDE=$PWD/build_variants/libfenv_prof.so timeout -k 10 100 python -u tools/ppo_phase_profile.py || exit $?
PAIRS=${PAIRS:-2} bash tools/ppo_ab.sh 2>&1 | sed -e "s/'workload'.*'us_per_minibatch'/us_per_minibatch/" -e "s/, 'samples_per_s.*//"
