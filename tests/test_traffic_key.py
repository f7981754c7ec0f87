"""The committed HBM-traffic measurement (profiles/traffic.json) belongs to
the kernel this tree benchmarks.

bench.py reports ``roofline.traffic`` only when its kernel_key (generated
assembly, leaf policy, compiled-program code, workload and programs) equals
the key the FETCH_SIZE / WRITE_SIZE passes ran under; a kernel change that
is not followed by a fresh tools/profile.sh run would otherwise leave the
bench line with ``traffic: null``.  CPU-only: the key is computed from the
generator and the compiled corpus, no GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench_env():
    """The environment a default bench run starts from (no layout knobs)."""
    env = dict(os.environ)
    for k in ("MYTHGPU_NREG", "MYTHGPU_LDS_SLOTS", "MYTHGPU_LIB"):
        env.pop(k, None)
    return env


def _run_json(code: str):
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=_bench_env(), check=True,
                         capture_output=True, text=True, timeout=600).stdout
    return json.loads(out.strip().splitlines()[-1])


def kernel_key_as_bench(workload: str, dags: int):
    """bench.kernel_key of a default ``bench.py --workload <workload>`` run,
    computed in a fresh process: the batch's register layout chosen as
    bench.py chooses it (mythril_amd/layout.py over the 16-slot programs)."""
    return _run_json(
        "import json, os, bench\n"
        "from mythril_amd import asmgen\n"
        "w = min(8, os.cpu_count() or 1)\n"
        "nreg, corpus = bench.choose_layout(bench.build_corpus(%d, w, workload=%r, nreg=16), w, "
        "None, %r)\n"
        "with asmgen.layout(nreg):\n"
        "    dg = asmgen.digest()\n"
        "print(json.dumps(bench.kernel_key(dg, %r, %d, 20, True, corpus, nreg)))\n"
        % (dags, workload, workload, workload, dags))


def test_bench_register_layouts():
    """the layout is chosen per batch from its 16-slot
    programs (mythril_amd/layout.py) — C2 runs the 11-slot, four-wave layout
    with five LDS regions, the query streams the 16-slot default with six
     — in ONE process, no import-time switch."""
    got = _run_json(
        "import json, os, bench\n"
        "from mythril_amd import layout\n"
        "from mythril_amd.engine import lds_slots_for\n"
        "out = {}\n"
        "for wl in ('c2', 'c3', 'c4', 'c5'):\n"
        "    c16 = bench.build_corpus(bench.default_units(wl), 8, workload=wl, nreg=16)\n"
        "    nreg, corpus = bench.choose_layout(c16, 8, None, wl)\n"
        "    assert all(p.nreg == nreg for _, p, _, _ in corpus)\n"
        "    ps = [p for _, p, _, _ in c16]\n"
        "    out[wl] = [nreg, lds_slots_for(nreg), layout.mean_scratch_slots(ps), "
        "layout.mean_heavy_share(ps)]\n"
        "print(json.dumps(out))\n")
    assert {w: v[:2] for w, v in got.items()} == {"c2": [11, 5], "c3": [16, 6], "c4": [16, 6],
                                                  "c5": [16, 6]}
    # C2: heavy arithmetic and few scratch spills; the streams: neither heavy
    assert got["c2"][2] <= layout_max_scratch() and got["c2"][3] >= 0.05
    assert all(got[w][3] < 0.01 for w in ("c3", "c4", "c5"))


def layout_max_scratch():
    from mythril_amd.layout import W4_MAX_SCRATCH_SLOTS
    return W4_MAX_SCRATCH_SLOTS


def test_traffic_json_keyed_to_this_tree():
    with open(os.path.join(ROOT, "profiles", "traffic.json")) as fh:
        tj = json.load(fh)
    entries = tj["entries"]
    key = kernel_key_as_bench("c2", 4096)
    c2 = [e for e in entries if e["kernel_key"].get("workload") == "c2"]
    assert c2, "profiles/traffic.json has no C2 entry"
    diff = sorted(k for k in key if c2[0]["kernel_key"].get(k) != key[k])
    assert not diff, "profiles/traffic.json is for another kernel (%s differ): " \
        "re-run tools/profile.sh + tools/prof_summary.py" % ", ".join(diff)
    for e in entries:
        # FETCH doubled (gfx950 correction) + WRITE, KiB -> bytes
        assert e["hbm_bytes_per_launch"] == (2 * e["fetch_kib"] + e["write_kib"]) * 1024
    # one entry per (workload, size, path)
    slots = [(e["kernel_key"]["workload"], e["kernel_key"]["dags"], e["kernel_key"]["jit"])
             for e in entries]
    assert len(slots) == len(set(slots))
