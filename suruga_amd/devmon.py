"""GPU clock and board power during a timed region, from sysfs (plain file
reads on a background thread, no subprocess, no GPU call).

bench.py prices its issue-bound roofline (valu_roofline) at the shader clock
the kernels actually ran at: MI355X sits at its board power cap under the C1
load, well below the 2.4 GHz peak clock.  The amdgpu driver
exposes, per card, hwmon `freq1_input` (sclk, Hz) and `power1_average` /
`power1_input` (uW), and `pp_dpm_sclk` (DPM levels, the current one marked
'*').  Whatever of these exists is sampled; missing files give None.
"""
from __future__ import annotations

import glob
import os
import threading
import time


def _read(path):
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return None


DRM = "/sys/class/drm"


def card_dirs(drm: str = DRM):
    """sysfs device directories of the amdgpu PCI functions (partition
    platform devices, amdgpu_xcp_*, carry no hwmon and are skipped)."""
    devs = []
    for d in sorted(glob.glob(os.path.join(drm, "card[0-9]*", "device"))):
        real = os.path.realpath(d)
        if real not in devs and (_read(os.path.join(d, "vendor")) or "").strip() == "0x1002" \
                and glob.glob(os.path.join(d, "hwmon", "hwmon*")):
            devs.append(real)
    return devs


def pick_card(pci_bus_id: str | None, drm: str = DRM):
    """(the card whose PCI address equals `pci_bus_id`, how it was chosen).
    A node has several cards, most of them another job's: without an exact
    match nothing is sampled unless exactly one card is visible."""
    devs = card_dirs(drm)
    if pci_bus_id:
        want = pci_bus_id.lower()
        for d in devs:
            if os.path.basename(d).lower() == want:
                return d, "pci address match"
    if len(devs) == 1:
        return devs[0], "only card visible"
    return None, f"no card with PCI address {pci_bus_id} among {len(devs)}"


class Sampler:
    """Samples sclk (MHz) and board power (W) of one card every `period` s
    between start() and stop()."""

    def __init__(self, pci_bus_id: str | None = None, period: float = 0.005, drm: str = DRM):
        self.period = period
        self.dev = None
        self.files = {}
        self.static = {}
        self.pci_bus_id = pci_bus_id
        d0, self.how = pick_card(pci_bus_id, drm)
        for d in ([d0] if d0 else []):
            self.dev = d
            for hw in sorted(glob.glob(os.path.join(d, "hwmon", "hwmon*"))):
                for key, name in (("sclk_hz", "freq1_input"), ("power_uw", "power1_average"),
                                  ("power_uw_in", "power1_input")):
                    p = os.path.join(hw, name)
                    if key not in self.files and os.path.exists(p):
                        self.files[key] = p
            if os.path.exists(os.path.join(d, "pp_dpm_sclk")):
                self.files["dpm"] = os.path.join(d, "pp_dpm_sclk")
            for hw in sorted(glob.glob(os.path.join(d, "hwmon", "hwmon*"))):
                for key, name in (("power_cap_w", "power1_cap"), ("power_label", "power1_label")):
                    v = _read(os.path.join(hw, name))
                    if v is not None and key not in self.static:
                        v = v.strip()
                        self.static[key] = int(v) / 1e6 if v.isdigit() else v
        self.samples = []
        self._stop = threading.Event()
        self._th = None

    def _one(self):
        s = {"t": time.perf_counter()}
        v = _read(self.files["sclk_hz"]) if "sclk_hz" in self.files else None
        if v and v.strip().isdigit():
            s["sclk_mhz"] = int(v) / 1e6
        elif "dpm" in self.files:
            for line in (_read(self.files["dpm"]) or "").splitlines():
                if line.strip().endswith("*"):
                    try:
                        s["sclk_mhz"] = float(line.split(":")[1].strip().rstrip("*").strip().lower().rstrip("mhz"))
                    except (IndexError, ValueError):
                        pass
        for key in ("power_uw", "power_uw_in"):
            v = _read(self.files[key]) if key in self.files else None
            if v and v.strip().isdigit():
                s["power_w"] = int(v) / 1e6
                break
        return s

    def _run(self):
        while not self._stop.is_set():
            self.samples.append(self._one())
            self._stop.wait(self.period)

    def start(self):
        if self.files:
            self._th = threading.Thread(target=self._run, daemon=True)
            self._th.start()
        return self

    def stop(self, t0=None, t1=None):
        self._stop.set()
        if self._th:
            self._th.join()
        return self.summary(t0, t1)

    def summary(self, t0=None, t1=None):
        """sclk: the samples taken in [t0, t1] (perf_counter; the timed region),
        its ramps at the edges dropped.  Power: the driver's power1_input is a
        running average over a window longer than a short timed region (it
        climbs from the idle value through the run), so the line reports its
        last value and maximum over the whole sampled span next to the
        region's mean."""
        inside = [s for s in self.samples if (t0 is None or s["t"] >= t0) and (t1 is None or s["t"] <= t1)]

        def stats(key, rows):
            v = [s[key] for s in rows if key in s]
            if not v:
                return None
            # drop the first and last tenth (ramps at the edges of the region)
            k = len(v) // 10
            core = v[k:len(v) - k] or v
            return {"mean": round(sum(core) / len(core), 1), "min": round(min(core), 1), "max": round(max(core), 1),
                    "samples": len(v)}

        pw = [s["power_w"] for s in self.samples if "power_w" in s]
        power = stats("power_w", inside)
        if power is not None and pw:
            power.update({"last": round(pw[-1], 1), "max_overall": round(max(pw), 1)})
        return {"card": self.dev, "pci_bus_id": self.pci_bus_id, "chosen_by": self.how,
                "sources": {k: os.path.basename(v) for k, v in self.files.items()},
                "sclk_mhz": stats("sclk_mhz", inside), "board_power_w": power, **self.static,
                "period_s": self.period}


def parse_cpulist(text: str) -> list[int]:
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]"""
    cpus = []
    for part in (text or "").strip().split(","):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        cpus.extend(range(int(lo), int(hi or lo) + 1))
    return cpus


def pin_to_gpu_node(pci_bus_id: str | None, drm: str = DRM):
    """Restrict the calling process to the CPUs of the GPU's own NUMA node
    (the card's `local_cpulist`, intersected with the CPUs it may use), so that
    host buffers first touched afterwards, and the record layer's copy threads
    created afterwards, sit next to the card's host link.  Without it a
    host-memory measurement lands on either socket of a two-socket host and
    its rate varies by tens of percent between runs.  Returns (cpus or None,
    how it was chosen); changes nothing when the card or its list is missing."""
    card, how = pick_card(pci_bus_id, drm)
    if card is None:
        return None, how
    local = set(parse_cpulist(_read(os.path.join(card, "local_cpulist")) or ""))
    allowed = set(os.sched_getaffinity(0))
    cpus = sorted(local & allowed)
    if not cpus:
        return None, "no CPU of the card's node is available to this process"
    os.sched_setaffinity(0, cpus)
    return cpus, f"{how}, NUMA-local CPUs"
