"""The command-line drop-ins run end to end: `python -m midaspom_amd` against
the compiled `midaspom` (MIDASPOM.out drop-in), and the torchrun form that
replaces `mpirun -np N MIDASPOM_MPI.out` (main_MIDASPOM_MPI.c:78,301,356,463,
479,484-506).  The torchrun test uses the gloo backend with both ranks on
cuda:0 (the launcher starts the rank processes before any GPU call); its
posterior file must equal the single-process file byte for byte (grid points
are independent, so the slab partition does not change a bit).  Nothing here
calls torch.cuda.synchronize(): the slab -> gather ordering is the engine's
stream contract."""
from __future__ import annotations

import os
import socket
import subprocess
import sys

import pytest

from midaspom_amd import _lib

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLAGS = ["-m", "400", "-d", "100", "-s", "101"]


def _env():
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    return env


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _strip_time(text):
    return [ln for ln in text.splitlines() if "Total running time" not in ln]


def test_python_cli_matches_compiled_cli(golden, tmp_path):
    # same relative output name in two directories: identical stdout too
    (tmp_path / "py").mkdir()
    (tmp_path / "c").mkdir()
    inp = str(golden / "occupancies.txt")
    rp = subprocess.run([sys.executable, "-m", "midaspom_amd", *FLAGS, "-g", "1", "-i", inp, "-o", "post.txt"],
                        capture_output=True, text=True, timeout=180, env=_env(), cwd=tmp_path / "py")
    assert rp.returncode == 0, rp.stderr
    rc = subprocess.run([str(_lib.CLI_PATH), *FLAGS, "-i", inp, "-o", "post.txt"],
                        capture_output=True, text=True, timeout=180, cwd=tmp_path / "c")
    assert rc.returncode == 0, rc.stderr
    assert (tmp_path / "py" / "post.txt").read_bytes() == (tmp_path / "c" / "post.txt").read_bytes()
    assert _strip_time(rp.stdout) == _strip_time(rc.stdout)
    assert "Total log-likelihood=-39.34251" in rp.stdout


def test_torchrun_cli_two_ranks(golden, tmp_path):
    single, multi = tmp_path / "single.txt", tmp_path / "multi.txt"
    inp = str(golden / "occupancies.txt")
    r1 = subprocess.run([sys.executable, "-m", "midaspom_amd", *FLAGS, "-i", inp, "-o", str(single)],
                        capture_output=True, text=True, timeout=180, env=_env(), cwd=ROOT)
    assert r1.returncode == 0, r1.stderr
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           "-m", "midaspom_amd", "--backend", "gloo", *FLAGS, "-i", inp, "-o", str(multi)]
    r2 = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r2.returncode == 0, r2.stderr[-3000:]
    assert multi.read_bytes() == single.read_bytes()
    out = r2.stdout
    # unguarded lines: once per rank (:78, :301, :356, :479)
    assert out.count("------ MIDASPOM, beta MPI version ------") == 2
    assert out.count("nextid=10\n") == 2
    for r in (1, 2):
        assert f"Starting parallel likelihood computation process {r}/2\n" in out
        assert f"end likelihood computation process {r}/2\n" in out
    # send / gather lines (:484-506); root-only progress over its 51 rows (:463)
    assert "Sending data (proc 1)... " in out and "Gathering data from 1 proc... " in out
    assert out.count("done\n") >= 4
    assert sum(1 for ln in out.splitlines() if ln.endswith("% done")) == 51
    assert out.count("Dispersal matrix:") == 1 and out.count("Total log-likelihood=-39.34251") == 1
    # (the ranks' lines interleave in the merged stdout: the per-rank order of
    # nextid after the dispersal matrix is checked in tests/test_cli_host.py)


def test_compiled_cli_slabs_round_robin_over_devices(golden, tmp_path):
    """-g 3 on a box with fewer GPUs: the three e-row slabs are dealt
    round-robin over the visible devices (one engine device context and
    stream each, main_MIDASPOM_MPI.c:361-368); the file equals -g 1's byte
    for byte.  MIDASPOM_TIMING=1 reports the wall-time split on stderr."""
    inp = str(golden / "config2_64x50.txt")
    outs = {}
    for g in ("1", "3"):
        out = tmp_path / f"g{g}.txt"
        r = subprocess.run([str(_lib.CLI_PATH), "-m", "400", "-d", "100", "-s", "203", "-g", g, "-i", inp,
                            "-o", str(out)], capture_output=True, text=True, timeout=180,
                           env=dict(os.environ, MIDASPOM_TIMING="1"))
        assert r.returncode == 0, r.stderr
        assert "midaspom timing (s): parse" in r.stderr and " write " in r.stderr
        outs[g] = out.read_bytes()
    assert outs["1"] == outs["3"]


def test_engine_several_contexts_one_device(golden):
    """mdp_loglik_grid over several device contexts (here all on device 0):
    the multi-device branch, slabs on their own streams, same result."""
    import numpy as np
    import midaspom_amd as mdp
    model = mdp.Model.load(golden / "config3_256x200.txt")
    g, _ = mdp.grid(157)
    with mdp.Engine(model, devices=[0]) as eng:
        one = eng.loglik_grid(g, g)
    with mdp.Engine(model, devices=[0, 0, 0, 0]) as eng:
        assert eng.info()["n_devices"] == 4
        four = eng.loglik_grid(g, g)
    assert np.array_equal(one, four)


@pytest.mark.parametrize("prog", ["midaspom_amd", "midaspom_amd.scenario", "midaspom_amd.future"])
def test_torchrun_one_rank_rccl(golden, tmp_path, prog):
    """`torchrun --nproc-per-node 1 ... --backend nccl` (the launcher starts
    the rank before any GPU call): RCCL initialises and the gather / reduce
    runs, as `mpirun -np 1 MIDASPOM_MPI.out` runs the MPI program; the file
    equals the single-process one byte for byte."""
    inp = str(golden / "occupancies.txt")
    if prog == "midaspom_amd":
        args = [*FLAGS]
    elif prog == "midaspom_amd.scenario":
        args = ["dieoff", *SCN_FLAGS["dieoff"]]
    else:
        post = tmp_path / "post.txt"
        r = subprocess.run([str(_lib.CLI_PATH), *FLAGS, "-i", inp, "-o", str(post)], capture_output=True, text=True,
                           timeout=180)
        assert r.returncode == 0, r.stderr
        args = ["-a", "20", "-m", "400", "-d", "100", "-q", str(post), "-n", "20000", "-r", "77"]
    single, multi = tmp_path / "single.txt", tmp_path / "multi.txt"
    r1 = subprocess.run([sys.executable, "-m", prog, *args, "-i", inp, "-o", str(single)],
                        capture_output=True, text=True, timeout=180, env=_env(), cwd=ROOT)
    assert r1.returncode == 0, r1.stderr
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           "-m", prog, *(args[:1] if prog.endswith("scenario") else []), "--backend", "nccl",
           *(args[1:] if prog.endswith("scenario") else args), "-i", inp, "-o", str(multi)]
    r2 = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r2.returncode == 0, r2.stderr[-3000:]
    assert multi.read_bytes() == single.read_bytes()
    assert "Gathering data from 0 proc... " in r2.stdout
    assert "process 1/1" in r2.stdout


SCN_FLAGS = {"dieoff": ["-a", "10", "-e", "0.3", "-c", "0.4", "-m", "400", "-d", "100", "-s", "21"],
             "loss": ["-a", "10", "-e", "0.3", "-c", "0.4", "-m", "400", "-d", "100", "-s", "13", "-v", "5"]}


def _scn_strip(text):
    return [ln for ln in text.splitlines() if "It took" not in ln]


@pytest.mark.parametrize("kind", ["dieoff", "loss"])
def test_python_scenario_cli_matches_compiled(golden, tmp_path, kind):
    """`python -m midaspom_amd.scenario` = the compiled midaspom_dieoff /
    midaspom_loss: same stdout lines, same file bytes."""
    (tmp_path / "py").mkdir()
    (tmp_path / "c").mkdir()
    inp = str(golden / "occupancies.txt")
    exe = _lib.DIEOFF_CLI_PATH if kind == "dieoff" else _lib.LOSS_CLI_PATH
    rp = subprocess.run([sys.executable, "-m", "midaspom_amd.scenario", kind, *SCN_FLAGS[kind], "-i", inp,
                         "-o", "lh.txt"], capture_output=True, text=True, timeout=180, env=_env(), cwd=tmp_path / "py")
    assert rp.returncode == 0, rp.stderr
    rc = subprocess.run([str(exe), *SCN_FLAGS[kind], "-i", inp, "-o", "lh.txt"], capture_output=True, text=True,
                        timeout=180, cwd=tmp_path / "c")
    assert rc.returncode == 0, rc.stderr
    assert (tmp_path / "py" / "lh.txt").read_bytes() == (tmp_path / "c" / "lh.txt").read_bytes()
    assert _scn_strip(rp.stdout) == _scn_strip(rc.stdout)


@pytest.mark.parametrize("kind", ["dieoff", "loss"])
def test_torchrun_scenario_two_ranks(golden, tmp_path, kind):
    """The MIDASPOM_{dieoff,loss}_MPI.out shape: K slabs over 2 ranks, one
    gather; the file equals the single-process one byte for byte."""
    inp = str(golden / "occupancies.txt")
    single, multi = tmp_path / "single.txt", tmp_path / "multi.txt"
    r1 = subprocess.run([sys.executable, "-m", "midaspom_amd.scenario", kind, *SCN_FLAGS[kind], "-i", inp,
                         "-o", str(single)], capture_output=True, text=True, timeout=180, env=_env(), cwd=ROOT)
    assert r1.returncode == 0, r1.stderr
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           "-m", "midaspom_amd.scenario", kind, "--backend", "gloo", *SCN_FLAGS[kind], "-i", inp, "-o", str(multi)]
    r2 = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r2.returncode == 0, r2.stderr[-3000:]
    assert multi.read_bytes() == single.read_bytes()
    out = r2.stdout
    assert out.count("beta MPI version") == 2
    for r in (1, 2):
        assert f"Starting parallel likelihood computation process {r}/2\n" in out
        assert f"end likelihood computation process {r}/2\n" in out
    assert "Sending data (proc 1)... " in out and "Gathering data from 1 proc... " in out
    assert out.count("Migration matrix:") == 1 and out.count("Writing on file") == 1


@pytest.mark.parametrize("kind", ["dieoff", "loss"])
def test_scenario_cli_multi_gpu_slabs(golden, tmp_path, kind):
    """-g N: the K grid in N slabs, one host thread + engine each (dealt
    round-robin over the visible GPUs, so N = 3 runs three engines on a
    one-GPU box concurrently); file bytes equal the -g 1 run, for the
    compiled CLI and the Python one.  N > s clamps to s slabs."""
    inp = str(golden / "occupancies.txt")
    exe = _lib.DIEOFF_CLI_PATH if kind == "dieoff" else _lib.LOSS_CLI_PATH
    outs = {}
    for tag, cmd in {"c1": [str(exe), "-g", "1"], "c3": [str(exe), "-g", "3"],
                     "c99": [str(exe), "-g", "99"],
                     "py3": [sys.executable, "-m", "midaspom_amd.scenario", kind, "-g", "3"]}.items():
        r = subprocess.run([*cmd, *SCN_FLAGS[kind], "-i", inp, "-o", str(tmp_path / f"{tag}.txt")],
                           capture_output=True, text=True, timeout=180, env=_env(), cwd=ROOT)
        assert r.returncode == 0, (tag, r.stderr[-2000:])
        outs[tag] = (tmp_path / f"{tag}.txt").read_bytes()
    assert outs["c3"] == outs["c1"] and outs["c99"] == outs["c1"] and outs["py3"] == outs["c1"]


# ---------------------------------------------------------------------------
# MIDASPOM_future: python -m midaspom_amd.future vs the compiled drop-in, the
# torchrun form of MIDASPOM_future_MPI.out, and -g N replicate ranges
# ---------------------------------------------------------------------------
FUT_FLAGS = ["-a", "20", "-m", "400", "-d", "100", "-S", "1", "-s", "200", "-n", "30001", "-r", "123"]


@pytest.fixture(scope="module")
def fut_post(tmp_path_factory, golden):
    import oracle  # the posterior the future program reads (CPU oracle, s = 101)

    p = tmp_path_factory.mktemp("fut") / "posterior.txt"
    oracle.run(golden / "occupancies.txt", p, m=400, d=100, s=101)
    return str(p)


def test_python_future_cli_matches_compiled(golden, tmp_path, fut_post):
    """Same stdout lines and file bytes (fixed seed) as the compiled
    midaspom_future."""
    (tmp_path / "py").mkdir()
    (tmp_path / "c").mkdir()
    inp = str(golden / "occupancies.txt")
    rp = subprocess.run([sys.executable, "-m", "midaspom_amd.future", *FUT_FLAGS, "-i", inp, "-q", fut_post,
                         "-o", "pext.txt"], capture_output=True, text=True, timeout=180, env=_env(),
                        cwd=tmp_path / "py")
    assert rp.returncode == 0, rp.stderr
    rc = subprocess.run([str(_lib.FUTURE_CLI_PATH), *FUT_FLAGS, "-i", inp, "-q", fut_post, "-o", "pext.txt"],
                        capture_output=True, text=True, timeout=180, cwd=tmp_path / "c")
    assert rc.returncode == 0, rc.stderr
    assert (tmp_path / "py" / "pext.txt").read_bytes() == (tmp_path / "c" / "pext.txt").read_bytes()
    assert _scn_strip(rp.stdout) == _scn_strip(rc.stdout)
    vals = [int(x) for x in (tmp_path / "c" / "pext.txt").read_text().split("\t")[:-1]]
    assert len(vals) == 20 and all(0 <= v <= 30001 for v in vals)


def test_torchrun_future_two_ranks(golden, tmp_path, fut_post):
    """The MIDASPOM_future_MPI.out shape: replicate ranges over 2 ranks, one
    sum-reduce; the file equals the single-process one byte for byte."""
    inp = str(golden / "occupancies.txt")
    single, multi = tmp_path / "single.txt", tmp_path / "multi.txt"
    r1 = subprocess.run([sys.executable, "-m", "midaspom_amd.future", *FUT_FLAGS, "-i", inp, "-q", fut_post,
                         "-o", str(single)], capture_output=True, text=True, timeout=180, env=_env(), cwd=ROOT)
    assert r1.returncode == 0, r1.stderr
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           "-m", "midaspom_amd.future", "--backend", "gloo", *FUT_FLAGS, "-i", inp, "-q", fut_post,
           "-o", str(multi)]
    r2 = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r2.returncode == 0, r2.stderr[-3000:]
    assert multi.read_bytes() == single.read_bytes()
    out = r2.stdout
    assert out.count("beta MPI version") == 1 and out.count("npstates = ") == 2
    for r in (1, 2):
        assert f"Starting parallel likelihood computation process {r}/2\n" in out
        assert f"end likelihood computation process {r}/2\n" in out
    assert "Sending data (proc 1)... " in out and "Gathering data from 1 proc... " in out
    assert out.count("Migration matrix:") == 1 and out.count("Writing on file") == 1


def test_future_cli_multi_gpu_ranges(golden, tmp_path, fut_post):
    """-g N: replicate ranges, one thread + engine each; the counts do not
    depend on N (addressed draws), for the compiled CLI and the Python one."""
    inp = str(golden / "occupancies.txt")
    outs = {}
    for tag, cmd in {"c1": [str(_lib.FUTURE_CLI_PATH), "-g", "1"], "c3": [str(_lib.FUTURE_CLI_PATH), "-g", "3"],
                     "py4": [sys.executable, "-m", "midaspom_amd.future", "-g", "4"]}.items():
        r = subprocess.run([*cmd, *FUT_FLAGS, "-i", inp, "-q", fut_post, "-o", str(tmp_path / f"{tag}.txt")],
                           capture_output=True, text=True, timeout=180, env=_env(), cwd=ROOT)
        assert r.returncode == 0, (tag, r.stderr[-2000:])
        outs[tag] = (tmp_path / f"{tag}.txt").read_bytes()
    assert outs["c3"] == outs["c1"] and outs["py4"] == outs["c1"]
