#!/bin/bash
# Run one gpurun call; when the pool reports it transient (nothing ran, nothing charged), wait and
# submit the same call again (up to N tries).  Any other outcome ends the loop.
N=${TRIES:-25}
for i in $(seq 1 $N); do
  out=$(/usr/local/graft/bin/gpurun "$@" 2>&1)
  rc=$?
  if echo "$out" | grep -q "status=transient"; then
    echo "[try $i] transient: $(echo "$out" | grep -o 'retry in [0-9]*s\|no free box\|busy' | head -1)"
    w=$(echo "$out" | grep -o 'retry in [0-9]*s' | grep -o '[0-9]*' | head -1)
    sleep $(( ${w:-90} + 15 ))
    continue
  fi
  echo "$out" | grep -v "every call sends"
  exit $rc
done
echo "gave up after $N transient tries"; exit 3
