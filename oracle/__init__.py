"""CPU oracle for the rray render path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this package.  It is the checker, never the thing measured or shipped:
the product (``rray_amd``) does not import it and has no CPU fallback.

``liboracle`` (rray_oracle.cpp) restates the reference Rust renderer
(/root/reference/src, snapshot 2024-08-07) op for op; ``scene_yaml`` restates
``scene_builder_yaml.rs`` on top of PyYAML (an independent YAML parser from the
product's C++ front-end), so a front-end bug on either side shows up as a
parity failure.
"""
from .oracle import Oracle, OracleCamera, build_oracle, lib_path  # noqa: F401
