"""Build librescore.so of another git revision into ab/<name>/ (an A/B of two builds in one GPU
session: RS_LIBRESCORE=ab/<name>/librescore.so selects it).  Usage: build_rev.py REV NAME"""
import importlib.util
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rev, name = sys.argv[1], sys.argv[2]
dst = os.path.join(REPO, "ab", name)
os.makedirs(dst, exist_ok=True)
tar = subprocess.run(["git", "-C", REPO, "archive", rev, "asr-rescoring_amd/csrc", "include"], check=True,
                     capture_output=True).stdout
subprocess.run(["tar", "-x", "-C", dst], input=tar, check=True)
spec = importlib.util.spec_from_file_location("_rs_build", os.path.join(REPO, "asr-rescoring_amd", "build.py"))
b = importlib.util.module_from_spec(spec)
spec.loader.exec_module(b)
print(b.build_library(verbose=True, csrc=os.path.join(dst, "asr-rescoring_amd", "csrc"),
                      out=os.path.join(dst, "librescore.so"), include=os.path.join(dst, "include")))
