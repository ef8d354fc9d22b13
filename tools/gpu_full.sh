# the whole GPU suite, then the counter list of this rocprofv3 (for PMC pass planning)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/full
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.txt 2>&1
rc=$?
echo "rc=$rc" >> $OUT/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
cd /tmp && timeout -k 10 60 rocprofv3 --list-avail > $OLDPWD/$OUT/counters.txt 2>&1 || true
