set -o pipefail
for s in 0 1 2 4 8 16 30 31; do echo -n "skip=$s "; HK_PCOND_SKIP=$s timeout -k 10 60 python3 tools/pcond_probe.py | tail -1 || exit 1; done
for s in 1 2 4 6; do echo -n "wide skip=$s "; HK_WIDE_SKIP=$s timeout -k 10 60 python3 tools/pcond_probe.py | tail -1 || exit 1; done
