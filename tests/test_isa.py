"""CPU: static ISA checks of the fence-free in-launch hand-offs. The beam step's batch-wide
stop test hands per-utterance flags to the utterance whose ticket add returns last without release /
acquire fences; that is valid on gfx950 only in the form MI355X_MICROARCH.md "Valid forms" row 1
measured: the flags stored write-through (sc1), the storing wave drained (vmcnt(0)) before its agent
atomic add, and the flags read back with sc1 loads. The parity tests cannot catch a compiler change that
drops a cache bit or moves the wait, so this test compiles k_beam.hip for gfx950 (device code only) and
checks the emitted instruction sequence of beam_step_kernel."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


def _kernel_asm(src, mangled_prefix, tmp_path):
    out = tmp_path / "k.s"
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-munsafe-fp-atomics",
                    "-S", "-o", str(out), os.path.join(ROOT, "whisper_context_biasing_amd", "csrc", src)],
                   check=True, capture_output=True, timeout=600)
    lines, body = out.read_text().splitlines(), None
    for i, ln in enumerate(lines):
        if ln.startswith(mangled_prefix) and ln.split(":")[0].startswith(mangled_prefix):
            body = []
            for ln2 in lines[i + 1:]:
                if ln2.startswith(".Lfunc_end"):
                    break
                body.append(ln2.strip())
            break
    assert body, f"{mangled_prefix} not found in {src}"
    return body


@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="hipcc not available")
def test_beam_step_flag_handoff_is_write_through_and_drained(tmp_path):
    body = _kernel_asm("k_beam.hip", "_ZN3wcb16beam_step_kernel", tmp_path)
    adds = [i for i, ln in enumerate(body) if ln.startswith("global_atomic_add ")]
    assert len(adds) == 1, adds                                   # the ticket
    a = adds[0]
    stores = [i for i, ln in enumerate(body[:a]) if re.match(r"global_store_dword\b.*\bsc1\b", ln)]
    assert len(stores) >= 2, "flag stores lost their sc1 (write-through) bit"
    assert any(body[j] == "s_waitcnt vmcnt(0)" for j in range(stores[-1] + 1, a)), \
        "no vmcnt(0) drain between the flag stores and the ticket add"
    loads = [ln for ln in body[a + 1:] if re.match(r"global_load_dword\b.*\bsc1\b", ln)]
    assert len(loads) >= 2, "the last arriver's flag loads lost their sc1 bit"
