# sourced by the round-6 GPU scripts: step NAME SECONDS cmd... runs one GPU step under its own
# time limit with its output in $O/NAME.out; a plain failure (rc 1-123) is recorded and the
# script goes on, a time limit / abort / signal (rc >= 124) ends the script there.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.out" 2>&1
  local rc=$?
  echo "step $n rc=$rc" >> "$O/steps.txt"
  if [ $rc -ne 0 ]; then tail -5 "$O/$n.out"; fi
  if [ $rc -ge 124 ]; then echo "stopping after $n (rc $rc)"; exit $rc; fi
  return 0
}
