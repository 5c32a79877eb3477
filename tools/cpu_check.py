import sys, os, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import bench
print(os.cpu_count(), open('/proc/cpuinfo').read().split('model name')[1].split('\n')[0])
for t, s in [(1, 5), (16, 20)]:
    print(bench.cpu_baseline(16, 48, 32768, t, s))
