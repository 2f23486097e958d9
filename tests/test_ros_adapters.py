"""CPU: the ROS node adapters compile.

``ros/src/pomdp/path_planning_2d_pp2.cpp`` and ``ros/src/mdp/path_planning_2d_pp2.cpp``
replace the reference's node classes (src/pomdp/path_planning_2d.cu:61-282,
src/mdp/path_planning_2d.cu:59-487) on top of include/pp2.h.  The image has no
ROS, Boost or OpenCV, so they are checked with ``g++ -fsyntax-only -Werror``
against the stand-in headers of tests/ros_stubs/ (the types and members the
adapters use, with the real libraries' signatures), the drop-in POMDP header
ros/include/path_planning_2d/pomdp_path_planning_2d.h first on the include
path, and the real pp2.h.  A wrong include, a misspelt pp2 call or a
signature mismatch with the node base class fails here instead of in a catkin
build.  (No link, no run: the node itself needs ROS.)
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUBS = os.path.join(ROOT, "tests", "ros_stubs")


@pytest.mark.parametrize("node", ["pomdp", "mdp"])
def test_ros_adapter_compiles(node):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    src = os.path.join(ROOT, "ros", "src", node, "path_planning_2d_pp2.cpp")
    cmd = [cxx, "-std=c++14", "-fsyntax-only", "-Wall", "-Wextra", "-Werror",
           "-Wno-unused-parameter",
           "-I", os.path.join(ROOT, "ros", "include"),
           "-I", STUBS, "-I", os.path.join(STUBS, "path_planning_2d"),
           "-I", os.path.join(ROOT, "include"), src]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
