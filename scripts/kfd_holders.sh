#!/bin/bash
# List the processes that hold the GPU (/dev/kfd) open, with their command lines (diagnostics for the
# box's per-GPU process limit).  Usage: scripts/kfd_holders.sh OUTFILE [DELAY_S]
sleep "${2:-60}"
for p in /proc/[0-9]*; do
  if ls -l "$p/fd" 2>/dev/null | grep -q "/dev/kfd"; then
    echo "$(basename "$p") $(tr '\0' ' ' < "$p/cmdline" | cut -c1-200)"
  fi
done > "$1"
