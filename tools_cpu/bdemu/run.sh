#!/bin/bash
# Host emulation of the NSGA-II fast path under AddressSanitizer + UBSan
# (VERDICT r5 item 5).  Builds the pre-deletion tree (cf1cf3a^, the last one
# with the m = 4 bitset kernels) and the working tree, then runs every case of
# make_cases.py through one dm_sort_nondominated call each:
#   pre, DM_BD_MAXM = 3 and 4 (the compare kernel / the bitset pass for M = 4),
#   worktree (the bitset pass and table-fed peel for M = 2, 3; compare for 4),
# with arenas filled with 0xC3 and with zeros (a fresh process's memory).
# Every line must read rc=0, 0 sanitizer reports, fronts == brute force.
set -u
cd "$(dirname "$0")"
python3 make_cases.py build/cases
make -s -j8 REV='cf1cf3a^' NAME=pre SAN=1 && make -s -j8 REV=worktree NAME=wt SAN=1 || exit 1
export ASAN_OPTIONS=detect_leaks=0 EMU_ALARM=900
one() {  # tag exe case [env...]
    local tag=$1 exe=$2 c=$3
    shift 3
    local r rc
    r=$(env "$@" timeout 1800 "$exe" "$c" 2>&1)
    rc=$?
    echo "$tag $(basename "$c") rc=$rc reports=$(echo "$r" | grep -c 'ERROR: AddressSanitizer\|runtime error\|check failed') $(echo "$r" | grep -E 'brute|golden' | tr '\n' ' ')"
}
for fill in 0xC3 0; do
    for c in build/cases/*.bin; do
        case $c in *m4_n4096*|*m4_n777*) slow=1 ;; *) slow=0 ;; esac
        one "pre maxm=4 fill=$fill" build/pre/harness_san "$c" EMU_BD_MAXM=4 EMU_ARENA_FILL=$fill
        [ $slow = 0 ] && one "pre maxm=3 fill=$fill" build/pre/harness_san "$c" EMU_BD_MAXM=3 EMU_ARENA_FILL=$fill
        [ $slow = 0 ] && one "wt fill=$fill" build/wt/harness_san "$c" EMU_ARENA_FILL=$fill
    done
done
