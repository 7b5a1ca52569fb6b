"""Run small JavaScript snippets in node (when installed) for differential tests."""
import json
import shutil
import subprocess

NODE = shutil.which("node") or shutil.which("nodejs")


def run_js(code: str, payload=None, timeout=60):
    """Evaluate ``code`` with ``const INPUT = <payload>``; the code must print to stdout."""
    src = f"const INPUT = {json.dumps(payload)};\n{code}\n"
    r = subprocess.run([NODE, "-e", src], capture_output=True, text=True, timeout=timeout)
    if r.returncode != 0:
        raise RuntimeError(r.stderr)
    return r.stdout
