#!/bin/bash
# Host-code sanitizer runs (CPU only, no GPU): the collective provider
# (lfa_coll*.c), the off_lfa provider and the multi-process peer-transport owner
# rebuilt with ASan+UBSan and with TSan, then examples/off_lfa_peer run with
# 2-3 ranks, owner-driven and progress-thread modes.  Kernels are not involved
# (the peer transport reduces on the host); liblfa.so is the normal build.
#   tools/sanitize_host.sh [outdir]      (default /tmp/lfa_sanitize)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
O=${1:-/tmp/lfa_sanitize}
FAB=${LFA_FABRIC_INCLUDE:-/root/reference/include}
for kind in asan tsan; do
  d=$O/$kind; mkdir -p "$d/out"
  if [ $kind = asan ]; then SAN="-fsanitize=address,undefined -fno-omit-frame-pointer -g -O1"
  else SAN="-fsanitize=thread -g -O1"; fi
  gcc $SAN -fPIC -std=gnu11 -Wall -D__HIP_PLATFORM_AMD__ -I"$R/include" -I/opt/rocm/include \
      -shared -o "$d/liblfa_coll.so" $(for f in lfa_coll lfa_coll_word lfa_coll_ws lfa_coll_host lfa_coll_group lfa_coll_exec; do echo "$R/libfabric_amd/csrc/$f.c"; done) "$R/libfabric_amd/csrc/lfa_coll_plan.c" "$R/libfabric_amd/csrc/lfa_coll_loopback.c" -L"$R/libfabric_amd" -llfa \
      -L/opt/rocm/lib -lamdhip64 -lrccl -lpthread -Wl,-rpath,"$R/libfabric_amd" -Wl,-soname,liblfa_coll.so
  gcc $SAN -fPIC -std=gnu11 -Wall -I"$R/include" -I"$FAB" -shared -o "$d/liboff_lfa-fi.so" \
      "$R/libfabric_amd/csrc/off_lfa.c" "$R/libfabric_amd/csrc/off_lfa_ep.c" -L"$d" -llfa_coll -L"$R/libfabric_amd" -llfa -lpthread -Wl,-rpath,'$ORIGIN'
  gcc $SAN -std=gnu11 -I"$R/include" -I"$FAB" -o "$d/peer" "$R/examples/off_lfa_peer.c" -ldl -lpthread
  for args in "3 manual" "3" "2 latency" "5 core" "4 core manual"; do
    set -- $args
    LD_LIBRARY_PATH="$R/libfabric_amd" timeout 300 "$d/peer" "$d/liboff_lfa-fi.so" "$1" "$d/out" \
        "${@:2}" 2>&1 | tee "$d/log.txt" | grep -E "^OK|^CORE broadcast|SUMMARY|WARNING" || true
    if grep -qE "SUMMARY|WARNING: ThreadSanitizer|ERROR: AddressSanitizer" "$d/log.txt"; then
      echo "$kind: sanitizer report (see $d/log.txt)"; exit 1
    fi
  done
done
echo "sanitizers clean"
