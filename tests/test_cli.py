"""yrt_raytrace, the drop-in for the reference's bin/raytrace (src/raytrace.cpp:256-287),
built over the C++ mirror include/yrt_raytrace.hpp."""
import subprocess

import numpy as np
import pytest

from helpers import ROOT, read_png_rgba8, scene_path

CLI = ROOT / "yocto_raytracing_amd" / "yrt_raytrace"


def run(*args, cwd=None):
    return subprocess.run([str(CLI), *map(str, args)], capture_output=True, text=True, cwd=cwd, timeout=300)


def test_cli_built():
    assert CLI.exists(), "build() must produce yocto_raytracing_amd/yrt_raytrace"


def test_cli_usage_errors():
    r = run("--bogus")
    assert r.returncode == 1 and "unknown option --bogus" in r.stderr
    r = run("-r")
    assert r.returncode == 1 and "missing value" in r.stderr
    r = run("-r", "abc", "x.obj")
    assert r.returncode == 1 and "bad value" in r.stderr
    assert run("--help").returncode == 0


def test_cli_missing_scene_fails_loudly(tmp_path):
    r = run(tmp_path / "missing.obj")
    assert r.returncode == 1
    assert "loading scene" in r.stdout and "cannot open" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("name,res,spp", [("simple", 72, 2), ("refl", 54, 1)])
def test_cli_renders_like_raytrace(tmp_path, name, res, spp):
    import yocto_raytracing_amd as yrt

    out = tmp_path / "out.png"
    r = run("-r", res, "-s", spp, "-o", out, scene_path(name))
    assert r.returncode == 0, r.stderr
    # the reference's messages, in order
    assert r.stdout.splitlines() == [f"loading scene {scene_path(name)}", "creating bvh", "tracing scene",
                                     f"saving image {out}"]
    s = yrt.load_scene(str(scene_path(name)))
    yrt.build_bvh(s)
    want = yrt.tonemap(yrt.raytrace(s, (0.1, 0.1, 0.1), res, spp))
    np.testing.assert_array_equal(read_png_rgba8(out), want)
