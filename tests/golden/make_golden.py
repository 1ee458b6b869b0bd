"""Regenerate tests/golden/ fixtures (run in the build container).

Provenance of every fixture (all are DATA -- inputs and expected outputs):
  occupancies.txt          copy of /root/reference/examples/input/occupancies.txt
                           (the reference's only shipped input; md5 d5306e9b...)
  manual_p3_obs.txt        the 3-year x 5-patch input of Manual_linux.pdf p.3 §3.1
  manual_p3_posterior.txt  the 5x5 posterior printed on Manual_linux.pdf p.3
                           (-m 400 -d 200 -s 5), 6 decimals
  anchors.json             reference outputs recorded in SURVEY.md §8(c) and
                           Appendix C (md5 of posterior files produced by the
                           reference in this container, Total log-likelihood
                           lines, argmax values) plus the manual's dieoff (p.4)
                           and loss (p.5) tables for the next rows of §8(f).
  config2_64x50.txt        synth.generate(**synth.CONFIG2)  (md5 6bd6f4bf...)
  config3_256x200.txt      synth.generate(**synth.CONFIG3)  (md5 5cf6ad09...)
  q1_64x50_mid.txt         synth.generate(**synth.Q1_MID): config 2 with the
                           variable block at columns 28-35, the SURVEY §8(c)
                           Q1 reproducer (its MPI-build Ltot is in anchors.json)
"""
import hashlib
import shutil
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parents[1]))
from midaspom_amd import synth  # noqa: E402

MANUAL_P3_OBS = "0 1 1 1 1\n0 -1 1 0 1\n1 0 1 1 0\n"
MANUAL_P3_POST = """0.000000 0.000000 0.000000 0.000000 0.000000
0.000000 0.612582 0.757902 0.374970 0.186856
0.000000 1.570907 2.757263 2.273996 1.547265
0.000000 0.844716 2.188557 2.634643 2.234809
0.000000 0.000000 0.000000 0.000000 0.000000
"""


def md5(p):
    return hashlib.md5(Path(p).read_bytes()).hexdigest()


def main():
    ref_in = Path("/root/reference/examples/input/occupancies.txt")
    if ref_in.exists():
        shutil.copyfile(ref_in, HERE / "occupancies.txt")
    (HERE / "manual_p3_obs.txt").write_text(MANUAL_P3_OBS)
    (HERE / "manual_p3_posterior.txt").write_text(MANUAL_P3_POST)
    synth.write(HERE / "config2_64x50.txt", **synth.CONFIG2)
    synth.write(HERE / "config3_256x200.txt", **synth.CONFIG3)
    synth.write(HERE / "q1_64x50_mid.txt", **synth.Q1_MID)
    assert md5(HERE / "config2_64x50.txt") == synth.MD5["config2"]
    assert md5(HERE / "config3_256x200.txt") == synth.MD5["config3"]
    assert md5(HERE / "occupancies.txt") == "d5306e9bbb6c873b4e38510f70a452c6"
    assert md5(HERE / "manual_p3_obs.txt") == "8859be5b77519bcf417664ad720b9024"
    print("fixtures written")


if __name__ == "__main__":
    main()
