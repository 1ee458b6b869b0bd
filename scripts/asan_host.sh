#!/bin/bash
# AddressSanitizer run of the host C code (parser, state enumeration, grid,
# normaliser, writers, CLIs) and of the C oracle, on the CPU test suite plus
# a random-input parser fuzz.  Works on a copy under /tmp; the in-tree build
# is untouched.  GPU code is not instrumented (no GPU sanitizers here).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/mdp_asan
rm -rf $W && mkdir -p $W
(cd $R && git ls-files | tar -cf - -T - | tar -xf - -C $W)
cp -r $R/midaspom_amd/_build $W/midaspom_amd/
rm -f $W/midaspom_amd/_build/spom_host.o $W/midaspom_amd/_build/spom_future_host.o $W/midaspom_amd/_build/libmidaspom.so \
      $W/midaspom_amd/_build/midaspom $W/midaspom_amd/_build/midaspom_dieoff $W/midaspom_amd/_build/midaspom_loss \
      $W/midaspom_amd/_build/midaspom_future
sed -i 's/^CFLAGS := -O2 -fPIC/CFLAGS := -O1 -g -fsanitize=address -fno-omit-frame-pointer -fPIC/' $W/midaspom_amd/csrc/Makefile
sed -i 's/^CFLAGS = -O2 -fPIC/CFLAGS = -O1 -g -fsanitize=address -fno-omit-frame-pointer -fPIC/' $W/oracle/Makefile
make -s -C $W/midaspom_amd/csrc -j8
make -s -C $W/oracle -j8
export LD_PRELOAD=$(gcc -print-file-name=libasan.so) ASAN_OPTIONS=detect_leaks=0
cd $W
python -m pytest tests -x -q -m "not gpu" -p no:cacheprovider
python - <<'PY'
import os, random, sys, tempfile
sys.path.insert(0, os.getcwd())
import midaspom_amd as mdp
rng = random.Random(1)
tokens = ["0", "1", "-1", " ", "\t", "\n", "2", "-", "x", "  ", "\r\n", "00", "1 1 1"]
ok = err = 0
p = os.path.join(tempfile.mkdtemp(), "f.txt")
for _ in range(1500):
    open(p, "w").write("".join(rng.choice(tokens) for _ in range(rng.randint(0, 60))))
    try:
        m = mdp.Model.load(p)
        _ = (m.npstates, m.prior, m.short_state)
        m.close()
        ok += 1
    except mdp.MidaspomError:
        err += 1
print(f"parser fuzz: {ok} parsed, {err} rejected, no sanitizer report")
PY
