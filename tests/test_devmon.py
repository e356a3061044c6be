"""suruga_amd.devmon on a synthetic sysfs tree (CPU): the card is chosen by
exact PCI address among several, partition devices without hwmon are
skipped, and the summary covers the samples of the given region."""
from __future__ import annotations

import os
import time

from suruga_amd import devmon


def _card(root, n, pci, sclk_hz, power_uw):
    dev = root / "devices" / pci
    hw = dev / "hwmon" / f"hwmon{n}"
    hw.mkdir(parents=True)
    (dev / "vendor").write_text("0x1002\n")
    (hw / "freq1_input").write_text(f"{sclk_hz}\n")
    (hw / "power1_input").write_text(f"{power_uw}\n")
    (hw / "power1_cap").write_text("1400000000\n")
    (root / "drm" / f"card{n}").mkdir(parents=True)
    os.symlink(dev, root / "drm" / f"card{n}" / "device")
    return hw


def test_sampler_picks_card_by_pci_address(tmp_path):
    _card(tmp_path, 0, "0000:75:00.0", 113_000_000, 241_000_000)
    hw = _card(tmp_path, 1, "0000:dc:00.0", 1_750_000_000, 1_390_000_000)
    xcp = tmp_path / "devices" / "amdgpu_xcp_0"  # a partition device: no hwmon
    xcp.mkdir(parents=True)
    (xcp / "vendor").write_text("0x1002\n")
    (tmp_path / "drm" / "card2").mkdir()
    os.symlink(xcp, tmp_path / "drm" / "card2" / "device")
    drm = str(tmp_path / "drm")
    assert len(devmon.card_dirs(drm)) == 2
    d, how = devmon.pick_card("0000:DC:00.0", drm)
    assert d.endswith("0000:dc:00.0") and how == "pci address match"
    assert devmon.pick_card("0000:01:00.0", drm)[0] is None  # no guessing among several cards
    s = devmon.Sampler("0000:dc:00.0", period=0.002, drm=drm).start()
    time.sleep(0.03)
    t0 = time.perf_counter()
    (hw / "freq1_input").write_text("1800000000\n")
    time.sleep(0.03)
    t1 = time.perf_counter()
    m = s.stop(t0, t1)
    assert m["chosen_by"] == "pci address match" and m["power_cap_w"] == 1400.0
    assert 1750.0 <= m["sclk_mhz"]["mean"] <= 1800.0 and m["sclk_mhz"]["max"] == 1800.0
    assert m["board_power_w"]["last"] == 1390.0


def test_sampler_without_card_reports_none(tmp_path):
    (tmp_path / "drm").mkdir()
    m = devmon.Sampler("0000:dc:00.0", drm=str(tmp_path / "drm")).start().stop()
    assert m["sclk_mhz"] is None and m["board_power_w"] is None and m["card"] is None


def test_parse_cpulist_and_pin_without_card(tmp_path):
    from suruga_amd import devmon

    assert devmon.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert devmon.parse_cpulist("") == []
    before = os.sched_getaffinity(0)
    cpus, how = devmon.pin_to_gpu_node("0000:aa:00.0", drm=str(tmp_path))  # no card: nothing changes
    assert cpus is None and os.sched_getaffinity(0) == before
