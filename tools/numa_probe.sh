echo "== cpus allowed"; grep -E "Cpus_allowed_list|Mems_allowed_list" /proc/self/status
echo "== lscpu"; lscpu | grep -iE "numa|socket|model name" 
echo "== gpu numa"; for d in /sys/class/drm/card*/device; do echo "$d $(cat $d/numa_node 2>/dev/null) $(cat $d/uevent 2>/dev/null | grep PCI_SLOT_NAME)"; done
echo "== rocm-smi bus"; timeout 30 rocm-smi --showbus 2>/dev/null | head -20
echo "== nodes"; ls /sys/devices/system/node/ | grep node; for n in /sys/devices/system/node/node*; do echo "$n $(cat $n/cpulist)"; done
