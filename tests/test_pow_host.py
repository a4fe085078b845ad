"""Host checks of the stepper's math (aigar_math.h, aigar_trig.h): the glibc pow
restatement against the C library's pow (which the reference's float power
calls), the exact non-negative fmod, and the correctly rounded trig."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_pow_glibc_matches_libm_pow(tmp_path):
    """aigar_math::pow_glibc == libm pow on 10^7 inputs (the path's masses,
    radii and cell counts, values near 1, random x over 2^+-40 and |y| <= 2):
    the device's fovSize and move speed round exactly like the reference's."""
    exe = str(tmp_path / "check_pow")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I",
                           os.path.join(ROOT, "aigar_amd", "csrc"), os.path.join(ROOT, "tools", "gen", "check_pow.cpp"),
                           "-o", exe])
    out = subprocess.run([exe, "10000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatches=0" in out.stdout, out.stdout


def test_mod_pos_matches_python_float_mod(tmp_path):
    """aigar_math::mod_pos (multiply + exact fma remainder) == Python's a % b
    for the non-negative offsets the grid footprints use (host build)."""
    exe = str(tmp_path / "check_mod")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I",
                           os.path.join(ROOT, "aigar_amd", "csrc"), os.path.join(ROOT, "tools", "gen", "check_mod.cpp"),
                           "-o", exe])
    out = subprocess.run([exe, "300000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatches=0" in out.stdout, out.stdout


def test_trunc_div_pos_matches_division(tmp_path):
    """aigar_math::trunc_div_pos (nearest integer of x * (1 / b) + an exact fma
    residual test) == int(x / b) on the observation's mask-loop operands and next
    to every k * b (host build; the device runs the same header)."""
    exe = str(tmp_path / "check_trunc_div")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I",
                           os.path.join(ROOT, "aigar_amd", "csrc"),
                           os.path.join(ROOT, "tools", "gen", "check_trunc_div.cpp"), "-o", exe])
    out = subprocess.run([exe, "300000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatches=0" in out.stdout, out.stdout


def test_trig_is_correctly_rounded(tmp_path):
    """aigar_trig.h sin_cr / cos_cr / atan2_cr == the quad-precision value
    rounded to double on the stepper's input shapes (host build).  glibc, which
    the reference runs, differs from that rounding on ~0.1% of them; OCML on
    4-27% (tools/micro/trig_vs_glibc.hip)."""
    exe = str(tmp_path / "check_trig")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I",
                           os.path.join(ROOT, "aigar_amd", "csrc"), os.path.join(ROOT, "tools", "gen", "check_trig.cpp"),
                           "-lquadmath", "-o", exe])
    out = subprocess.run([exe, "100000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatches=0 " in out.stdout, out.stdout
    glibc = float(out.stdout.split("(")[1].split("%")[0])
    assert glibc < 0.5, out.stdout


def test_pellet_radius_constants():
    """aigar_sem.h folds the radii of 1-, 2- and 3-mass pellets (cell.py:210-212)
    to constants: they must be Python's math.sqrt(m / math.pi) exactly."""
    import math
    import re
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "aigar_amd", "csrc", "aigar_sem.h")).read()
    consts = dict(re.findall(r"kPelletR(\d) = (0x[0-9a-fp.+-]+)", hdr))
    assert sorted(consts) == ["1", "2", "3"]
    for m, c in consts.items():
        assert float.fromhex(c) == math.sqrt(int(m) / math.pi), m


def test_glibc_trig_matches_libm(tmp_path):
    """aigar_glibc_trig.h sin / cos / atan2 == the C library's (which the reference's math
    module calls) on ~11 M inputs shaped like the path's (host build); where the static libm
    is present, also == its FMA variants __sin_fma / __cos_fma / __ieee754_atan2_fma, linked
    directly.  -fno-builtin-*: gcc would otherwise fuse sin(a), cos(a) into sincos(), a
    different glibc routine (oracle/Makefile does the same)."""
    exe = str(tmp_path / "check_glibc_trig")
    cmd = ["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-builtin-sin", "-fno-builtin-cos",
           "-fno-builtin-atan2", "-I", os.path.join(ROOT, "aigar_amd", "csrc"),
           os.path.join(ROOT, "tools", "gen", "check_glibc_trig.cpp"), "-o", exe]
    libm_a = "/usr/lib/x86_64-linux-gnu/libm-2.35.a"
    if os.path.exists(libm_a):
        objs = ["s_sin-fma.o", "e_atan2-fma.o", "sincostab.o", "branred.o"]
        subprocess.check_call(["ar", "x", libm_a] + objs, cwd=str(tmp_path))
        cmd[1:1] = ["-DAIGAR_LINK_FMA_VARIANTS"]
        cmd += [str(tmp_path / o) for o in objs]
    subprocess.check_call(cmd)
    out = subprocess.run([exe, "5000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatches=0" in out.stdout, out.stdout
