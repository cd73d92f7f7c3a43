"""ISA checks of the fused MLP kernels (CPU: hipcc cross-compiles gfx950).

The kernels read MFMA fragments from LDS with inline-asm ds_read_b128 and wait
for them explicitly; the compiler assumes the destination registers are written
when the asm issues. If it reuses one before the drain (e.g. because it deleted
a consumer MFMA whose result it proved dead), the late LDS data clobbers a live
value -- an address, in the fault that motivated this test. Also pins the MFMA
count (no slice's work folded away) and zero scratch.

Round 5: the checker walked the control-flow graph from the file's first
block only, i.e. it checked the first kernel of each .s (mlp_x3_clock_kernel,
mlp_fused_kernel) and none of the others; it now starts from every kernel's
entry, so the inference, training, backward, weight-gradient and layer kernels
are all held to it (tools/check_async_lds.py).
"""
import os
import re
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "nerf-rep_for_test_amd")
sys.path.insert(0, os.path.join(REPO, "tools"))

pytestmark = pytest.mark.skipif(not shutil.which("/opt/rocm/bin/hipcc") and
                                not shutil.which("hipcc"), reason="hipcc not available")

# (file, kernel symbol, MFMA mnemonic, count in that kernel's body): fp32:
# 2 + 10 + 4x(128) + 64 slices' worth; x3: 792 = (2 + 8 + 2) x 48 (layer loop
# body once) + 4 x 48 + 24
KERNELS = [("mlp_fused.s", "mlp_fused_kernel", "v_mfma_f32_16x16x4_f32", 2112),
           ("mlp_x3.s", "mlp_x3_kernel", "v_mfma_f32_16x16x32_f16", 792)]


def kernel_body(text, symbol):
    """The .s text of one kernel: from its label to its .Lfunc_end marker."""
    m = re.search(r"^(_ZN7nerfhip\d+" + symbol + r"\w*):", text, re.M)
    assert m, symbol
    end = text.index(".Lfunc_end", m.end())
    return text[m.start():end]


@pytest.fixture(scope="module")
def asm_dir():
    subprocess.run(["make", "-C", PKG, "-s", "asm-mlp"], check=True, capture_output=True,
                   timeout=600)
    return os.path.join(PKG, "build", "asm")


@pytest.mark.parametrize("name,symbol,mfma,count", KERNELS)
def test_no_async_lds_hazard(asm_dir, name, symbol, mfma, count):
    import check_async_lds
    assert check_async_lds.main(os.path.join(asm_dir, name)) == 0


@pytest.mark.parametrize("name,symbol,mfma,count", KERNELS)
def test_mfma_count_and_no_scratch(asm_dir, name, symbol, mfma, count):
    text = open(os.path.join(asm_dir, name)).read()
    body = kernel_body(text, symbol)
    assert len(re.findall(r"^\s+" + mfma + r"\b", body, re.M)) == count
    # no kernel in the file spills
    assert not re.search(r"\.private_segment_fixed_size:\s+[1-9]", text)
