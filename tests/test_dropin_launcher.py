"""bgx_main.py (the src/main.py drop-in launcher): the reference's main.py
and the worker processes it spawns import THIS build's `multi` package, not
the reference's (which sits next to main.py and would win under a plain
`python src/main.py`). A stand-in reference tree with a decoy `multi`
package and main.py's process structure (spawn start method, worker
Process, main.py:2, 86-91, 163-169) checks it on CPU."""
import os
import subprocess
import sys
import textwrap

from conftest import PKG

MAIN = textwrap.dedent('''
    import multiprocessing
    import multi

    def worker_function(q):
        import multi as m
        q.put(m.__file__)

    if __name__ == "__main__":
        try:
            multiprocessing.set_start_method("spawn")
        except RuntimeError:
            pass
        q = multiprocessing.Queue()
        p = multiprocessing.Process(target=worker_function, args=(q,))
        p.start()
        print("PARENT", multi.__file__)
        print("CHILD", q.get(timeout=120))
        p.join()
''')


def test_launcher_puts_the_build_ahead_of_the_reference(tmp_path):
    src = tmp_path / "src"
    (src / "multi").mkdir(parents=True)
    (src / "multi" / "__init__.py").write_text("raise ImportError('the reference multi package was imported')\n")
    (src / "main.py").write_text(MAIN)
    env = dict(os.environ)
    env.pop("PYTHONPATH", None)
    r = subprocess.run([sys.executable, os.path.join(PKG, "bgx_main.py"), str(src / "main.py")],
                       capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = dict(ln.split(" ", 1) for ln in r.stdout.strip().splitlines() if ln.split(" ")[0] in ("PARENT", "CHILD"))
    want = os.path.join(PKG, "multi", "__init__.py")
    assert os.path.realpath(lines["PARENT"]) == os.path.realpath(want)
    assert os.path.realpath(lines["CHILD"]) == os.path.realpath(want)
