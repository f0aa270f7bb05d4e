"""setuptools hook: compile the native core, HIP kernels (gfx950) and CLI in-tree before packaging."""
import subprocess
import sys
from pathlib import Path

from setuptools import setup
from setuptools.command.build_py import build_py


class BuildNative(build_py):
    def run(self):
        subprocess.check_call([sys.executable, str(Path(__file__).parent / "tools" / "build.py")])
        super().run()


setup(cmdclass={"build_py": BuildNative})
