#!/usr/bin/env python3
"""Why the bench's engine scan (fls_scan_* into pinned host memory, bench.py
e2e_rates) runs ~300 M rows/s in some processes and ~195 in others (round 6,
profiles/r6/abe2e3_r6ai/): one fresh process per run, each printing where its
pinned host buffers live (NUMA node of the pages, move_pages), the node of
the CPUs it may run on, the GPU's node, a plain hipMemcpy D2H rate into a
hipHostMalloc buffer, and the engine scan's rate (best of 3 passes, as the
bench).

    python scripts/e2e_numa.py --runs 4 [--scale 10]
"""
import argparse
import ctypes as C
import glob
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def page_nodes(addrs):
    """NUMA node of the page holding each address (-errno when unknown)."""
    libc = C.CDLL(None, use_errno=True)
    n = len(addrs)
    pages = (C.c_void_p * n)(*[a & ~4095 for a in addrs])
    status = (C.c_int * n)()
    rc = libc.syscall(C.c_long(279), C.c_int(0), C.c_ulong(n), pages, None, status, C.c_int(0))
    return [int(s) for s in status] if rc == 0 else [f"move_pages rc {rc} errno {C.get_errno()}"]


def smaps_of(addrs):
    """For each address: its mapping's size, AnonHugePages, KernelPageSize and
    file (hipHostMalloc memory may be anonymous or a device mapping)."""
    maps, cur = [], None
    with open("/proc/self/smaps") as f:
        for ln in f:
            parts = ln.split()
            if "-" in parts[0] and len(parts) >= 5 and not parts[0].endswith(":"):
                lo, hi = (int(x, 16) for x in parts[0].split("-"))
                cur = {"lo": lo, "hi": hi, "file": parts[5] if len(parts) > 5 else ""}
                maps.append(cur)
            elif cur is not None and parts[0] in ("AnonHugePages:", "KernelPageSize:", "Rss:", "THPeligible:"):
                cur[parts[0][:-1]] = " ".join(parts[1:])
    out = set()
    for a in addrs:
        for m in maps:
            if m["lo"] <= a < m["hi"]:
                out.add(f"{(m['hi'] - m['lo']) >> 20} MB rss {m.get('Rss')} thp {m.get('AnonHugePages')} "
                        f"kps {m.get('KernelPageSize')} elig {m.get('THPeligible')} {m['file']}")
    return sorted(out)


def host_state():
    res = {}
    for f in ("/sys/kernel/mm/transparent_hugepage/enabled", "/sys/kernel/mm/transparent_hugepage/defrag"):
        try:
            res[os.path.basename(f)] = Path(f).read_text().strip()
        except OSError:
            pass
    try:
        mi = dict(ln.split(":", 1) for ln in Path("/proc/meminfo").read_text().splitlines())
        res["meminfo"] = {k: mi[k].strip() for k in ("MemFree", "MemAvailable", "AnonHugePages", "Cached") if k in mi}
    except OSError:
        pass
    try:  # free blocks per order (0..10) on each node's Normal zone
        res["buddy"] = [ln.split()[1] + ":" + ",".join(ln.split()[4:]) for ln in
                        Path("/proc/buddyinfo").read_text().splitlines() if "Normal" in ln]
    except OSError:
        pass
    return res


def cpu_nodes():
    out = {}
    for cpu in sorted(os.sched_getaffinity(0)):
        nodes = glob.glob(f"/sys/devices/system/cpu/cpu{cpu}/node*")
        nd = int(os.path.basename(nodes[0])[4:]) if nodes else -1
        out[nd] = out.get(nd, 0) + 1
    return out


class LinkSampler:
    """Samples the GPU's PCIe link state (sysfs, read-only) every 5 ms; phase()
    labels what runs, and summary() counts the distinct states seen per phase."""

    def __init__(self, busid):
        import threading
        d = Path(f"/sys/bus/pci/devices/{busid}").resolve()
        self.files = [f for f in (d / "current_link_speed", d / "current_link_width", d / "pp_dpm_pcie", d / "pp_dpm_socclk",
                                  d / "pp_dpm_fclk", d / "pp_dpm_mclk", d / "pp_dpm_sclk") if f.exists()]
        # the links above it (a switch between the GPU and the root port)
        for up in list(d.parents)[:4]:
            f = up / "current_link_speed"
            if f.exists():
                self.files.append(f)
        self.label, self.seen, self.stop = "idle", {}, False
        self.th = threading.Thread(target=self.run, daemon=True)
        self.th.start()

    def read(self):
        out = []
        for f in self.files:
            try:
                v = f.read_text().strip()
            except OSError as e:
                v = f"err {e.errno}"
            if f.parent.name != self.files[0].parent.name:
                v = f"{f.parent.name}={v}"
            if f.name.startswith("pp_dpm_"):  # the active level is marked '*'
                v = f.name[7:] + " " + (" ".join(ln for ln in v.splitlines() if "*" in ln) or v.replace("\n", "|"))
            out.append(v)
        return " / ".join(out)

    def run(self):
        while not self.stop:
            k = (self.label, self.read())
            self.seen[k] = self.seen.get(k, 0) + 1
            time.sleep(0.005)

    def phase(self, label):
        self.label = label

    def summary(self):
        self.stop = True
        self.th.join()
        return {f"{lab}: {st}": n for (lab, st), n in self.seen.items()}


def child(a):
    sys.path.insert(0, str(ROOT))
    import pkgload
    fl = pkgload.load()
    hip = C.CDLL("libamdhip64.so")
    bus = C.create_string_buffer(64)
    hip.hipDeviceGetPCIBusId(bus, 64, 0)
    busid = bus.value.decode().lower()
    try:
        gpu_node = int(Path(f"/sys/bus/pci/devices/{busid}/numa_node").read_text())
    except OSError:
        gpu_node = None
    res = {"pid": os.getpid(), "cpu_nodes": cpu_nodes(), "gpu_bus": busid, "gpu_node": gpu_node}
    res["host"] = host_state()
    ls = LinkSampler(busid)
    # control: a plain D2H into one hipHostMalloc buffer
    nb = 1 << 30
    h, d = C.c_void_p(), C.c_void_p()
    hip.hipHostMalloc(C.byref(h), C.c_size_t(nb), 0)
    hip.hipMalloc(C.byref(d), C.c_size_t(nb))
    hip.hipMemset(d, 1, C.c_size_t(nb))
    hip.hipMemcpy(h, d, C.c_size_t(nb), 2)
    best = 0
    ls.phase("d2h")
    for _ in range(3):
        t0 = time.perf_counter()
        hip.hipMemcpy(h, d, C.c_size_t(nb), 2)
        best = max(best, nb / (time.perf_counter() - t0) / 1e9)
    res["d2h_gbs_hostmalloc"] = round(best, 1)
    ls.phase("h2d")
    best = 0
    for _ in range(3):
        t0 = time.perf_counter()
        hip.hipMemcpy(d, h, C.c_size_t(nb), 1)
        best = max(best, nb / (time.perf_counter() - t0) / 1e9)
    res["h2d_gbs_hostmalloc"] = round(best, 1)
    res["hostmalloc_nodes"] = sorted(set(page_nodes([h.value + i * (nb // 16) for i in range(16)])), key=str)
    res["hostmalloc_smaps"] = smaps_of([h.value])
    hip.hipHostFree(h)
    hip.hipFree(d)
    ls.phase("gen")
    img = fl.gen_image("lineitem_full", a.scale, 0, 0, None, 16)
    t = fl.Connection([0]).read_image(img)
    for _ in t.scan():
        break
    out = fl.RowGroup()
    passes, nodes, sc_addrs = [], set(), []
    for p in range(3):
        ls.phase(f"scan{p}")
        rows = 0
        t0 = time.perf_counter()
        fl._check(fl.lib.fls_scan_begin(t.h, None, 0, t.nrowgroups))
        while fl._check(fl.lib.fls_scan_next(t.h, C.byref(out))) == 1:
            rows += out.nrows
            if p == 0 and out.rowgroup % 16 == 0:
                cols = [out.columns[c] for c in range(out.ncols) if out.columns[c]]
                nodes.update(page_nodes(cols))
                sc_addrs += cols
        passes.append(rows / (time.perf_counter() - t0))
    res["engine_rows_s"] = [round(x / 1e6, 1) for x in passes]
    res["scan_buffer_nodes"] = sorted(nodes, key=str)
    res["scan_buffer_smaps"] = smaps_of(sc_addrs)
    res["link"] = ls.summary()
    t.close()
    img.close()
    print(json.dumps(res), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=4)
    ap.add_argument("--scale", type=float, default=10)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--arms", default="default:", help="name:K=V,K=V;name2:... environments, alternated per run")
    ap.add_argument("--brief", action="store_true", help="print the rates only")
    a = ap.parse_args()
    if a.child:
        child(a)
        return
    arms = []
    for spec in a.arms.split(";"):
        name, _, kv = spec.partition(":")
        arms.append((name, dict(x.split("=", 1) for x in kv.split(",") if x)))
    for r in range(a.runs):
        for name, env in arms:
            p = subprocess.run([sys.executable, __file__, "--child", "--scale", str(a.scale)], capture_output=True,
                               text=True, timeout=300, env={**os.environ, **env})
            if p.returncode != 0:
                print(p.stderr[-2000:], file=sys.stderr)
                sys.exit(p.returncode)
            line = p.stdout.strip().splitlines()[-1]
            if a.brief:
                d = json.loads(line)
                line = (f"d2h {d['d2h_gbs_hostmalloc']} h2d {d['h2d_gbs_hostmalloc']} GB/s, engine {d['engine_rows_s']} "
                        f"M rows/s")
            print(f"run {r} {name}: {line}", flush=True)


if __name__ == "__main__":
    main()
