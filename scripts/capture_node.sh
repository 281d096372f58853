#!/usr/bin/env bash
# Capture this node's GPU-facing sysfs/devfs facts into a directory tree that
# libmxnode can read back with --root (used to build tests/fixtures/sysfs/real_*).
# Only small text attributes are copied; nothing is written outside $OUT.
set -u
OUT=${1:-gpurun_out/node_capture}
mkdir -p "$OUT"
TOPO=/sys/class/kfd/kfd/topology
if [ -d $TOPO ]; then
  find $TOPO -type f -not -path "*/caches/*" 2>/dev/null | while read -r f; do
    mkdir -p "$OUT$(dirname "$f")"
    timeout 2 cat "$f" > "$OUT$f" 2>/dev/null || true
  done
fi
for bdf in $(cat $TOPO/nodes/*/properties 2>/dev/null | awk '$1=="location_id"{print $2}' | sort -u); do :; done
for d in /sys/bus/pci/devices/*; do
  v=$(cat "$d/vendor" 2>/dev/null); c=$(cat "$d/class" 2>/dev/null)
  if [ "$v" = "0x1002" ] && [ "${c:0:4}" = "0x12" -o "${c:0:4}" = "0x03" ]; then
    mkdir -p "$OUT$d"
    for a in vendor device class numa_node subsystem_device revision current_link_speed current_link_width; do
      timeout 2 cat "$d/$a" > "$OUT$d/$a" 2>/dev/null || true
    done
    if [ -d "$d/drm" ]; then for e in $(ls "$d/drm"); do mkdir -p "$OUT$d/drm/$e"; done; fi
  fi
done
mkdir -p "$OUT/dev/dri"
ls -l /dev/dri /dev/kfd > "$OUT/dev_listing.txt" 2>&1 || true
for n in /dev/dri/*; do [ -e "$n" ] && : > "$OUT$n"; done
[ -e /dev/kfd ] && : > "$OUT/dev/kfd"
ls -la /sys/class/drm > "$OUT/sys_class_drm.txt" 2>&1 || true
id > "$OUT/id.txt" 2>&1
tar -C "$OUT" -czf "$OUT.tar.gz" . && rm -rf "$OUT"
echo "captured into $OUT.tar.gz"
