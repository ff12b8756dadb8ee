"""The device state a bench line ran on: HIP device attributes plus what the box's own
amd-smi reports for clocks, power cap, partition modes and memory -- read-only queries, each under a time limit.

    from tools.device_state import device_state
    d = device_state(0)              # dict, JSON-serialisable; missing tools give None fields, never raise

`python tools/device_state.py [--full]` prints it (--full adds the raw amd-smi JSON under "raw").
"""
import ctypes
import json
import os
import subprocess
import sys

# hipDeviceAttribute_t values of ROCm 7.2 (hip_runtime_api.h; printed by a one-line C program against the header)
_ATTR = {'clock_khz': 5, 'mem_clock_khz': 60, 'pci_bus': 67, 'cu_count': 63, 'mem_bus_bits': 59, 'pci_domain': 69}


def _hip_attrs(dev):
    try:
        lib = ctypes.CDLL('libamdhip64.so')
    except OSError:
        try:
            lib = ctypes.CDLL('/opt/rocm/lib/libamdhip64.so')
        except OSError:
            return None
    out = {}
    for k, a in _ATTR.items():
        v = ctypes.c_int(0)
        if lib.hipDeviceGetAttribute(ctypes.byref(v), ctypes.c_int(a), ctypes.c_int(dev)) == 0:
            out[k] = v.value
    return out


def _smi_json(args, timeout=25):
    try:
        p = subprocess.run(['amd-smi'] + args + ['--json'], capture_output=True, text=True, timeout=timeout)
    except (OSError, subprocess.SubprocessError):
        return None
    if p.returncode != 0:
        return None
    try:
        return json.loads(p.stdout)
    except ValueError:
        return None


def _first_gpu(j):
    """amd-smi --json output: a list of per-GPU dicts (or {'gpu_data': [...]} in some versions)."""
    if isinstance(j, dict):
        j = j.get('gpu_data', j)
    if isinstance(j, list) and j:
        return j[0]
    return j if isinstance(j, dict) else None


def _val(d, *path):
    for p in path:
        if not isinstance(d, dict) or p not in d:
            return None
        d = d[p]
    if isinstance(d, dict) and 'value' in d:
        return '%s %s' % (d['value'], d.get('unit', '')) if d.get('unit') else d['value']
    return d


def device_state(dev=0, full=False):
    """HIP attributes of `dev` (as the process sees it) + amd-smi's view of the visible GPU: clocks (current sclk /
    mclk / fclk), power (current, cap), compute / memory partition mode, VRAM use, temperature, throttle status."""
    out = {'hip': _hip_attrs(dev)}
    try:
        import torch
        if torch.cuda.is_available():
            p = torch.cuda.get_device_properties(dev)
            out['name'] = p.name
            out['arch'] = getattr(p, 'gcnArchName', None)
            out['total_mem_gib'] = round(p.total_memory / 2 ** 30, 1)
    except Exception:   # measurement metadata: never fail the bench over it
        pass
    out['visible'] = os.environ.get('HIP_VISIBLE_DEVICES') or os.environ.get('ROCR_VISIBLE_DEVICES')
    met = _first_gpu(_smi_json(['metric']))
    sta = _first_gpu(_smi_json(['static']))
    part = _first_gpu(_smi_json(['partition'], timeout=15))
    smi = {}
    if met:
        clk = met.get('clock') or {}
        for name in ('gfx_0', 'mem_0', 'fclk_0', 'socclk_0'):
            c = clk.get(name)
            if isinstance(c, dict):
                smi[name + '_mhz'] = _val(c, 'clk')
                if name == 'gfx_0':
                    smi['gfx_0_max_mhz'] = _val(c, 'max_clk')
        pw = met.get('power') or {}
        smi['power_w'] = _val(pw, 'socket_power')
        smi['power_cap'] = _val(met, 'power', 'power_limit') or _val(met, 'power_cap')
        smi['temp_hotspot'] = _val(met, 'temperature', 'hotspot')
        smi['temp_mem'] = _val(met, 'temperature', 'mem')
        smi['vram_used'] = _val(met, 'mem_usage', 'used_vram')
        smi['throttle'] = met.get('throttle') if isinstance(met.get('throttle'), (dict, str)) else None
        smi['usage'] = met.get('usage')
    if sta:
        smi['bus'] = _val(sta, 'bus', 'bdf')
        smi['vbios'] = _val(sta, 'vbios', 'version')
        smi['driver'] = _val(sta, 'driver', 'version')
        smi['power_cap_static'] = _val(sta, 'limit', 'max_power') or _val(sta, 'limit', 'ppt0', 'max_power_limit')
        smi['static_partition'] = sta.get('partition')
        smi['vram'] = sta.get('vram')
    if part:
        smi['partition'] = part
    out['smi'] = smi or None
    if full:
        out['raw'] = {'metric': met, 'static': sta, 'partition': part}
    return out


class PowerWindow:
    """Power / clock / throttle residency of the GPU over a window (bench.py's timed region), read in-process through
    the amdsmi library (sysfs gpu_metrics; microseconds per read, nothing on the GPU's queues):

        w = PowerWindow(dev); w.start(); ...timed launches...; w.mid(); ...; info = w.stop()

    -> avg_power_w (energy counter delta / wall), ppt_residency (fraction of the window the package power limit was
    throttling: delta ppt_residency_acc / delta accumulation_counter), thermal residencies, mean gfx clock over the
    XCDs at mid(), average umc / gfx activity, hotspot / HBM temperature at stop. Every field is None where the
    library or the field is absent; nothing raises."""

    def __init__(self, dev=0):
        self.h = None
        self.m0 = self.m1 = None
        self.mids = []
        try:
            import amdsmi
            self.smi = amdsmi
            amdsmi.amdsmi_init()
            hs = amdsmi.amdsmi_get_processor_handles()
            bus = (_hip_attrs(dev) or {}).get('pci_bus')
            for h in hs:
                bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)
                if bus is None or int(bdf.split(':')[1], 16) == bus:
                    self.h, self.bdf = h, bdf
                    break
        except Exception:
            self.h = None

    def _read(self):
        if self.h is None:
            return None
        try:
            m = self.smi.amdsmi_get_gpu_metrics_info(self.h)
            e = self.smi.amdsmi_get_energy_count(self.h)
            import time
            return dict(m=m, e=e, t=time.perf_counter())
        except Exception:
            return None

    def start(self):
        self.m0 = self._read()

    def mid(self):
        r = self._read()
        if r is not None:
            self.mids.append(r)

    @staticmethod
    def _num(x):
        return x if isinstance(x, (int, float)) and not isinstance(x, bool) else None

    def stop(self):
        self.m1 = self._read()
        a, b = self.m0, self.m1
        if a is None or b is None:
            return None
        out = {'bdf': self.bdf, 'window_s': b['t'] - a['t']}
        try:
            de = (b['e']['energy_accumulator'] - a['e']['energy_accumulator']) * b['e']['counter_resolution'] * 1e-6
            out['avg_power_w'] = de / out['window_s'] if out['window_s'] > 0 else None
        except Exception:
            out['avg_power_w'] = None
        ma, mb = a['m'], b['m']
        acc = [self._num(ma.get('accumulation_counter')), self._num(mb.get('accumulation_counter'))]
        for k in ('ppt_residency_acc', 'socket_thm_residency_acc', 'hbm_thm_residency_acc', 'prochot_residency_acc',
                  'vr_thm_residency_acc'):
            x0, x1 = self._num(ma.get(k)), self._num(mb.get(k))
            ok = None not in (x0, x1, *acc) and acc[1] > acc[0]
            out[k.replace('_acc', '')] = (x1 - x0) / (acc[1] - acc[0]) if ok else None
        for k in ('average_umc_activity', 'average_gfx_activity', 'average_socket_power', 'average_gfxclk_frequency',
                  'average_uclk_frequency', 'temperature_hotspot', 'temperature_mem', 'temperature_hbm',
                  'throttle_status', 'indep_throttle_status'):
            v = mb.get(k)
            out[k] = v if isinstance(v, (int, float, str)) else None
        per = []   # per mid() sample: the XCDs' current gfx clocks
        for r in (self.mids or [b]):
            c = [x for x in (r['m'].get('current_gfxclks') or []) if self._num(x) and x < 0xFFFF]
            if c:
                per.append(c)
        out['gfxclk_mhz_mean'] = sum(map(sum, per)) / sum(map(len, per)) if per else None
        out['gfxclk_mhz_min'] = min(map(min, per)) if per else None
        out['gfxclk_samples'] = len(per)
        out['uclk_mhz'] = self._num((self.mids or [b])[-1]['m'].get('current_uclk'))
        return out


if __name__ == '__main__':
    print(json.dumps(device_state(0, full='--full' in sys.argv), default=str, indent=1))
