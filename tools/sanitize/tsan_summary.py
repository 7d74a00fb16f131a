"""Classify a ThreadSanitizer log of tools/sanitize/host_stress (SANITIZER=tsan run).

  python tools/sanitize/tsan_summary.py gpurun_out/tsan_r04.log

For every report: data races by the module of the racing access's first frame,
lock-order cycles by whether every mutex lock in them is called from the HIP /
HSA runtimes.  A report that names this repo's code (elect_amd/csrc, include/,
tools/sanitize) in those positions is listed in full."""
import re
import sys
from collections import Counter

OURS = ("elect_amd/csrc", "include/elect", "tools/sanitize", "host_path", "ec_capi", "rs_kernels", "libec_jni")
RUNTIMES = ("libamdhip64", "libhsa-runtime64")


def frame_module(line: str) -> str:
    m = re.search(r"\((\S+?)\+0x[0-9a-f]+\)", line)
    if m:
        return m.group(1).split("/")[-1]
    m = re.search(r" (/\S+):\d+", line)
    return m.group(1) if m else line.strip()[:60]


def main(path):
    text = open(path, errors="replace").read()
    reports = text.split("==================")
    races, cycles, ours = Counter(), [0, 0], []
    for r in reports:
        if "WARNING: ThreadSanitizer: data race" in r:
            # the racing access's first frame outside TSan's own interceptors (new/delete, mutex)
            frames = []
            for l in r.splitlines()[1:]:
                if not re.match(r"\s+#\d+ ", l):
                    if frames:
                        break
                    continue
                frames.append(l)
            first = next((l for l in frames if "compiler-rt/lib/tsan" not in l), frames[0] if frames else "")
            mod = frame_module(first)
            races[mod] += 1
            if any(o in first for o in OURS):
                ours.append(r.strip())
        elif "lock-order-inversion" in r:
            cycles[0] += 1
            locks = [l for l in r.splitlines() if "pthread_mutex_lock" in l or "Mutex" in l]
            callers = []
            lines = r.splitlines()
            for i, l in enumerate(lines):
                if re.match(r"\s+#0 pthread_mutex_lock", l) and i + 1 < len(lines):
                    callers.append(lines[i + 1])
            if callers and all(any(rt in c for rt in RUNTIMES) for c in callers):
                cycles[1] += 1
            elif any(any(o in c for o in OURS) for c in callers):
                ours.append(r.strip())
    print(f"data races: {sum(races.values())}; racing access by module: {dict(races)}")
    print(f"lock-order cycles: {cycles[0]}; every lock called from the HIP/HSA runtimes: {cycles[1]}")
    print(f"reports naming this repo's code first: {len(ours)}")
    for r in ours[:5]:
        print("-----\n" + r[:3000])


if __name__ == "__main__":
    main(sys.argv[1])
