"""GPU clock / power / temperature telemetry through amdsmi (fail-soft).

Benchmarks on a shared pool vary by +-5 % from box to box and run to run; the clocks and power the GPU ran at
during the timed region tell throttling apart from a software regression. ``GpuTelemetry(device_index)``
resolves the amdsmi handle of a HIP device by PCI bus id; ``start()`` samples in a background thread,
``stop()`` returns min / mean / max per field. Every amdsmi call is guarded: without the library, a driver or
permission, the summary is simply empty.
"""
from __future__ import annotations

import threading
from typing import Dict, List, Optional


def _amdsmi():
    try:
        import amdsmi  # type: ignore

        amdsmi.amdsmi_init()
        return amdsmi
    except Exception:
        return None


def _bdf_of(device_index: int) -> Optional[str]:
    """PCI address of a HIP device (amdsmi may list GPUs that HIP_VISIBLE_DEVICES hides, so indices differ)."""
    try:
        import torch

        if not torch.cuda.is_available():
            return None
        p = torch.cuda.get_device_properties(device_index)
        return "%04x:%02x:%02x" % (getattr(p, "pci_domain_id", 0), p.pci_bus_id, p.pci_device_id)
    except Exception:
        return None


class GpuTelemetry:
    def __init__(self, device_index: int = 0):
        self.smi = _amdsmi()
        self.handle = None
        self._samples: List[Dict[str, float]] = []
        self._stop = threading.Event()
        self._th: Optional[threading.Thread] = None
        if self.smi is None:
            return
        try:
            handles = self.smi.amdsmi_get_processor_handles()
            want = _bdf_of(device_index)
            for h in handles:
                bdf = str(self.smi.amdsmi_get_gpu_device_bdf(h)).lower()
                if want is not None and bdf.startswith(want):
                    self.handle = h
                    break
            if self.handle is None and want is None and len(handles) == 1:
                self.handle = handles[0]
        except Exception:
            self.handle = None

    @property
    def ok(self) -> bool:
        return self.handle is not None

    def sample(self) -> Dict[str, float]:
        if self.handle is None:
            return {}
        smi, h, out = self.smi, self.handle, {}
        try:
            out["gfx_mhz"] = float(smi.amdsmi_get_clock_info(h, smi.AmdSmiClkType.GFX)["clk"])
        except Exception:
            pass
        try:
            out["mem_mhz"] = float(smi.amdsmi_get_clock_info(h, smi.AmdSmiClkType.MEM)["clk"])
        except Exception:
            pass
        try:
            pw = smi.amdsmi_get_power_info(h)
            for k in ("current_socket_power", "average_socket_power", "socket_power"):
                v = pw.get(k)
                if isinstance(v, (int, float)) and v > 0:
                    out["power_w"] = float(v)
                    break
        except Exception:
            pass
        try:
            out["hotspot_c"] = float(smi.amdsmi_get_temp_metric(h, smi.AmdSmiTemperatureType.HOTSPOT,
                                                               smi.AmdSmiTemperatureMetric.CURRENT))
        except Exception:
            pass
        return out

    def start(self, period_s: float = 0.2) -> None:
        if self.handle is None:
            return
        self._samples = [self.sample()]
        self._stop.clear()

        def loop():
            while not self._stop.wait(period_s):
                self._samples.append(self.sample())

        self._th = threading.Thread(target=loop, daemon=True)
        self._th.start()

    def stop(self) -> Dict[str, Dict[str, float]]:
        if self._th is not None:
            self._stop.set()
            self._th.join(timeout=2)
            self._th = None
        if self.handle is not None:
            self._samples.append(self.sample())
        return summarize(self._samples)


def summarize(samples: List[Dict[str, float]]) -> Dict[str, Dict[str, float]]:
    keys = sorted({k for s in samples for k in s})
    out = {}
    for k in keys:
        v = [s[k] for s in samples if k in s]
        out[k] = {"min": round(min(v), 1), "mean": round(sum(v) / len(v), 1), "max": round(max(v), 1), "n": len(v)}
    return out
