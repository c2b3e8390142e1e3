"""Pins the CPU oracle (oracle/rt_oracle.c) before it is trusted as the parity checker.

  * tests/golden/eigen_kat.bin: every Eigen 3.3.7 float expression of the hot path, evaluated by the
    reference's vendored Eigen (oracle/eigen_kat.cpp) -- the oracle must reproduce every bit;
  * tests/golden/tucano_kat.bin: the camera (getCenter, screenToWorld) and model-matrix
    (normalizeModelMatrix) known answers computed by the reference's own Tucano code, compiled
    unmodified (oracle/tucano_kat.cpp, no GL library linked);
  * tests/golden/survey_kat.json: values printed by the unmodified reference at survey time
     -- ray directions (bits), hit distances, colours, box counts and the
    per-pass box sequence of generateBoundingBoxes.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, scene_path


def _read_kat_file(name):
    raw = open(os.path.join(GOLDEN, name), "rb").read()
    magic, count = np.frombuffer(raw[:8], np.uint32)
    assert magic == 0x4B54414B
    off, secs = 8, []
    for _ in range(count):
        op, n, il, ol = (int(x) for x in np.frombuffer(raw[off:off + 16], np.int32))
        off += 16
        inp = np.frombuffer(raw[off:off + 4 * n * il], np.float32).copy()
        off += 4 * n * il
        exp = np.frombuffer(raw[off:off + 4 * n * ol], np.float32).copy()
        off += 4 * n * ol
        secs.append((op, n, il, ol, inp, exp))
    return secs


def read_kat():
    """Known answers: the Eigen expressions from eigen_kat.bin (the reference's vendored Eigen), with the
    camera / model-matrix ops (SHAPE 8, CENTER 15, SCREEN 16) taken from tucano_kat.bin -- computed by the
    reference's own Tucano::Camera / Tucano::Model code (oracle/tucano_kat.cpp)."""
    tucano = {s[0]: s for s in _read_kat_file("tucano_kat.bin")}
    return [tucano.get(s[0], s) for s in _read_kat_file("eigen_kat.bin")]


def test_tucano_kat_from_reference_code_equals_eigen_kat():
    """The reference's Tucano::Camera::getCenter / screenToWorld and Model::normalizeModelMatrix (compiled
    unmodified, oracle/tucano_kat.cpp) give exactly the bits of eigen_kat.cpp's restated formulas, on the
    same 2,000 inputs per op."""
    eig = {s[0]: s for s in _read_kat_file("eigen_kat.bin")}
    tuc = _read_kat_file("tucano_kat.bin")
    assert sorted(s[0] for s in tuc) == [8, 15, 16]
    for op, n, il, ol, inp, exp in tuc:
        e = eig[op]
        assert (n, il, ol) == e[1:4] and inp.tobytes() == e[4].tobytes()
        assert exp.view(np.uint32).tolist() == e[5].view(np.uint32).tolist(), op


def same_bits(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    return (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))


@pytest.mark.parametrize("sec", read_kat(), ids=lambda s: f"op{s[0]}")
def test_oracle_eigen_primitives_bit_exact(orc, sec):
    op, n, il, ol, inp, exp = sec
    got = orc.kat(op, inp, n, ol)
    bad = (~same_bits(got, exp)).reshape(n, ol).any(1)
    assert bad.sum() == 0, f"{orc.KAT_OPS[op]}: {bad.sum()} / {n} cases differ from Eigen"


def bits(v):
    return ["%08x" % x for x in np.asarray(v, np.float32).view(np.uint32)]


@pytest.mark.parametrize("key", ["cube", "dodge"])
def test_oracle_matches_reference_known_answers(orc, key):
    kat = json.load(open(os.path.join(GOLDEN, "survey_kat.json")))[key]
    mesh = orc.Mesh.load_obj(scene_path(kat["scene"]))
    scene = orc.Scene(mesh)
    assert scene.box_count() == kat["boxes"]
    if "pass_counts" in kat:
        assert scene.pass_counts() == kat["pass_counts"]
    W, H = kat["W"], kat["H"]
    cam = orc.flycam(W, H)
    for px in kat["pixels"]:
        i, j = px["ij"]
        o, d = orc.camera_ray(cam, i, j)
        assert bits(d) == px["dir"], (i, j)
        rgb, face, t = scene.render(cam, orc.DEFAULT_LIGHTS, W, H, full=True, pixels=[(i, j)])
        if px.get("miss"):
            assert face[0] == -1 and np.isinf(t[0])
            np.testing.assert_array_equal(rgb[0], np.float32(0.9))
        else:
            assert np.float32(t[0]) == np.float32(px["t"])
            np.testing.assert_array_equal(rgb[0], np.array(px["rgb"], np.float32))


def test_oracle_bunny_box_count(orc):
    kat = json.load(open(os.path.join(GOLDEN, "survey_kat.json")))["bunny"]
    mesh = orc.Mesh.load_obj(scene_path("bunny.obj"))
    assert mesh.counts()[1] == kat["n_faces"]
    assert orc.Scene(mesh).box_count() == kat["boxes"]


def test_oracle_golden_images(orc):
    """Oracle output is stable against the committed golden images (tests/golden/images.npz)."""
    g = np.load(os.path.join(GOLDEN, "images.npz"))
    for key in g.files:
        if not key.endswith("_rgb"):
            continue
        name = key[:-4]
        scene_name, mode, W, H = name.split("__")
        W, H = int(W), int(H)
        mesh = orc.Mesh.load_obj(scene_path(scene_name + ".obj"))
        sc = orc.Scene(mesh)
        cam = orc.flycam(W, H)
        rgb, face, t = sc.render(cam, orc.DEFAULT_LIGHTS, W, H, full=(mode == "full"), threads=8)
        np.testing.assert_array_equal(rgb.reshape(H, W, 3), g[name + "_rgb"])
        np.testing.assert_array_equal(face.reshape(H, W), g[name + "_face"])
