#!/bin/bash
# Shader clock and power of the visible GPU while a bench runs (diagnostic: is the seal
# power-limited?).  Samples `amd-smi metric` (or rocm-smi) every ~0.25 s into <out>.clk
# while the command runs.   bash tools/clock_watch.sh <out> <command...>
out=$1; shift
( while true; do
    date +%s.%N
    if command -v amd-smi > /dev/null; then
      amd-smi metric -c -p 2>/dev/null | grep -E -A1 "SOCKET_POWER|GFX_0:" | grep -E "SOCKET_POWER|CLK:" | head -2
    else
      rocm-smi --showclocks --showpower 2>/dev/null | grep -E -i "sclk|power" | head -4
    fi
    sleep 0.25
  done ) > $out.clk 2>&1 &
w=$!
"$@"
rc=$?
kill $w 2>/dev/null
wait $w 2>/dev/null
exit $rc
