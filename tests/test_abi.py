"""CPU tests of the drop-in boundary: libyavo.so loads and exports every symbol include/yavo/*.h declares,
the record layouts are byte-identical to the reference's KeyPoint / Matches, and the product never routes
through the oracle or a CPU path.  No compute calls are made (no GPU here)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import ya_vo_amd as yv

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", "yavo", h) for h in ("yavo.h", "yavo_types.h", "yavo_geom.h",
                                                                       "yavo_io.h", "yavo_map.h")]


def _declared_functions():
    names = set()
    for h in HEADERS:
        if not os.path.exists(h):
            continue
        txt = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(yv_\w+)\s*\(", txt, flags=re.M):
            names.add(m.group(1))
    return names


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(yv.LIB_PATH):
        subprocess.run(["make", "-C", os.path.join(ROOT, "ya_vo_amd", "csrc"), "-j8"], check=True)
    return yv.load_library()


def test_every_declared_symbol_is_exported(lib):
    declared = _declared_functions()
    assert len(declared) >= 20
    for name in sorted(declared):
        assert hasattr(lib, name), f"{name} declared in include/yavo but not exported"
        assert any(name in t for t in (yv.SIGNATURES, yv.GEOM_SIGNATURES, yv.IO_SIGNATURES, yv.MAP_SIGNATURES)), \
            f"{name} has no ctypes binding"


def test_abi_version_and_status_strings(lib):
    assert lib.yv_abi_version() == 2
    assert lib.yv_status_string(0) == b"ok"
    assert lib.yv_status_string(-3) == b"no usable GPU"


def test_record_layout_matches_reference_classes(tmp_path):
    # compile a probe against the public header: offsets must equal the numpy dtypes (and KeyPoint/Matches)
    src = tmp_path / "probe.c"
    src.write_text(
        '#include <stddef.h>\n#include <stdio.h>\n#include "yavo/yavo_types.h"\n'
        "int main(void){printf(\"%zu %zu %zu %zu %zu %zu %zu %zu\\n\", sizeof(yv_keypoint), offsetof(yv_keypoint,id),"
        " offsetof(yv_keypoint,matched), offsetof(yv_keypoint,featVec), sizeof(yv_match), offsetof(yv_match,pt2),"
        " offsetof(yv_match,distance), offsetof(yv_keypoint,y));return 0;}\n")
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    vals = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert vals == [48, 8, 12, 13, 100, 48, 96, 4]
    kd, md = yv.KEYPOINT_DTYPE, yv.MATCH_DTYPE
    assert (kd.itemsize, kd.fields["id"][1], kd.fields["matched"][1], kd.fields["featVec"][1]) == (48, 8, 12, 13)
    assert (md.itemsize, md.fields["pt2"][1], md.fields["distance"][1]) == (100, 48, 96)


def test_batch_view_layout_matches_ctypes(tmp_path):
    # the ctypes mirror of yv_batch_view must agree with the C compiler field by field
    fields = [f for f, _ in yv._BatchView._fields_]
    src = tmp_path / "probe_view.c"
    body = " ".join(f'printf("%zu ", offsetof(yv_batch_view, {f}));' for f in fields)
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "yavo/yavo.h"\n'
                   f'int main(void){{{body} printf("%zu\\n", sizeof(yv_batch_view)); return 0;}}\n')
    exe = tmp_path / "probe_view"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    vals = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    expect = [getattr(yv._BatchView, f).offset for f in fields] + [ctypes.sizeof(yv._BatchView)]
    assert vals == expect


def test_no_device_means_error_not_fallback(lib):
    if lib.yv_device_count() > 0:
        pytest.skip("a GPU is visible; the no-device path is exercised on CPU boxes only")
    h = ctypes.c_void_p()
    assert lib.yv_create(0, ctypes.byref(h)) == yv.YV_ERR_NODEVICE
    with pytest.raises(yv.YavoError):
        yv.Context(0)


def test_invalid_arguments_rejected_without_device(lib):
    # argument validation happens before any device work
    n = ctypes.c_int()
    assert lib.yv_detect(None, None, 10, 10, 10, 10, None, None, ctypes.byref(n), None) == yv.YV_ERR_INVALID
    assert lib.yv_batch_create(None, 1, 376, 1241, 2000, 1, ctypes.byref(ctypes.c_void_p())) == yv.YV_ERR_INVALID


def test_product_never_touches_the_oracle():
    for dirpath, _, files in os.walk(os.path.join(ROOT, "ya_vo_amd")):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp", ".cc", "Makefile")):
                txt = open(os.path.join(dirpath, f), errors="ignore").read()
                assert "liboracle" not in txt and "oracle_bind" not in txt and "or_fast_detect" not in txt, f


def test_library_has_gfx950_code_object():
    # the fat binary embeds an offload bundle whose target id names gfx950
    blob = open(yv.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
