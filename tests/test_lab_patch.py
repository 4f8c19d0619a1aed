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


def _kernels(asm):
    """Kernel name -> instruction lines (comments dropped) of a device .s."""
    out = {}
    for m in re.finditer(r"^(_Z\w+):.*$", asm, re.M):
        end = asm.find(".Lfunc_end", m.end())
        out[m.group(1)] = [re.sub(r"\s*;.*$", "", ln) for ln in asm[m.end():end].split("\n")
                           if ln.strip() and not ln.strip().startswith(";")]
    return out


def test_lab_default_build_is_the_product(tmp_path):
    """With no variant macro set, the patched sources compile to the
    product's kernels instruction for instruction, so an A/B against a lab
    variant differs only by its macro (round 6: a define the pruning had
    dropped left the lab's default build without record stores, 11 % faster
    than the product for the wrong reason)."""
    hipcc = "/opt/rocm/bin/hipcc"
    if not (shutil.which("patch") and os.path.exists(hipcc)):
        pytest.skip("no patch tool or hipcc")
    dst = tmp_path / "src"
    shutil.copytree(os.path.join(ROOT, "zero-packet_amd", "csrc"), dst / "zero-packet_amd" / "csrc")
    shutil.copytree(os.path.join(ROOT, "include"), dst / "include")
    with open(os.path.join(ROOT, "tools", "patches", "lab.patch")) as f:
        subprocess.run(["patch", "-s", "-p1", "-d", str(dst)], stdin=f, check=True)
    # every macro a lab #if tests is defined somewhere (an undefined one reads as 0)
    lab = dst / "zero-packet_amd" / "csrc"
    text = "".join(open(os.path.join(lab, f)).read() for f in os.listdir(lab)
                   if f.endswith((".hip", ".h")))
    for name in ("zp_parse.hip", "zp_stream.h", "zp_build.hip", "zp_ctx.hip"):
        for m in re.finditer(r"^\s*#\s*(?:el)?if\s+(.*)$", open(lab / name).read(), re.M):
            expr = re.sub(r"defined\s*\(?\s*\w+\s*\)?", "", m.group(1))
            for ident in re.findall(r"\b([A-Z_][A-Z0-9_]+)\b", expr):
                assert re.search(r"#\s*define\s+" + ident + r"\b", text), (name, ident)
    jobs = {}
    for tag, root in (("product", CSRC), ("lab", str(lab))):
        for src in ("zp_parse.hip", "zp_parse_slots.hip", "zp_build.hip"):
            out = str(tmp_path / f"{tag}_{src}.s")
            jobs[(tag, src)] = (out, subprocess.Popen(
                [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                 "--cuda-device-only", "-S", "-o", out, os.path.join(root, src)],
                stdout=subprocess.DEVNULL, stderr=subprocess.PIPE))
    for out, p in jobs.values():
        assert p.wait(timeout=600) == 0, p.stderr.read()
    for src in ("zp_parse.hip", "zp_parse_slots.hip", "zp_build.hip"):
        a = _kernels(open(jobs[("product", src)][0]).read())
        b = _kernels(open(jobs[("lab", src)][0]).read())
        assert a and set(a) == set(b), src
        for k in a:
            assert a[k] == b[k], (src, k)
