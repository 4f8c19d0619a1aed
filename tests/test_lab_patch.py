"""CPU: the product kernels carry no variant or ablation branches, and the
lab patch that puts them back for A/B builds (tools/patches/lab.patch,
applied by tools/build_variants.sh to a scratch copy) still applies to the
current sources."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "zero-packet_amd", "csrc")
LAB_ONLY = ("ZP_ABL_", "ZB_ABL_", "ZP_STAMPS", "ZB_STAMPS", "ZP_ONE_STAMPS", "ZP_DBG_FBCOUNT",
            "ZP_FB2", "ZP_SUMW_BYTES", "ZP_REC_PLAIN", "ZP_SEG", "ZP_NO_PRIO", "ZP_NO_TAIL",
            "ZP_REGION", "ZP_CSUM_MOD", "ZP_FMASK_ITEM", "ZB_NO_SECTOR_WB", "ZB_PIPE_SEARCH",
            "ZB_LANE_PAY", "ZB_SKIP_PAY", "ZB_OP_PREFETCH")


@pytest.mark.parametrize("name", ["zp_parse.hip", "zp_stream.h", "zp_build.hip", "zp_ctx.hip"])
def test_product_has_no_variant_branches(name):
    text = open(os.path.join(CSRC, name)).read()
    conds = re.findall(r"^\s*#\s*(?:if|ifdef|ifndef|elif)\b.*$", text, re.M)
    bad = [c for c in conds if any(k in c for k in LAB_ONLY)]
    assert not bad, bad


def test_lab_patch_applies(tmp_path):
    if not shutil.which("patch"):
        pytest.skip("no patch tool")
    dst = tmp_path / "src"
    shutil.copytree(os.path.join(ROOT, "zero-packet_amd", "csrc"), dst / "zero-packet_amd" / "csrc")
    shutil.copytree(os.path.join(ROOT, "include"), dst / "include")
    with open(os.path.join(ROOT, "tools", "patches", "lab.patch")) as f:
        r = subprocess.run(["patch", "-p1", "--dry-run", "-d", str(dst)], stdin=f,
                           capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "FAILED" not in r.stdout and "fuzz" not in r.stdout, r.stdout
