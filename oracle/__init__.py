"""TEST INFRASTRUCTURE ONLY — the CPU oracle of the detect -> match -> pose hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this package, and only as the *checker* (or the timed CPU baseline).  The product path
(``thor-slam_amd/``) never imports it and fails loudly when its HIP library is missing.

Parity status: the reference's hot path runs inside the closed cuVSLAM binary
(``launch/thor_visual_slam.launch.py:30-33``), which is absent from ``/root/reference``, so
**parity against cuVSLAM itself is unpinned**.  This oracle is the NumPy restatement of the
algorithm the build defines for rows A2-A7 of SURVEY.md §8a.  What *is* pinned against the
reference's own code (run in the build container, vectors committed under ``tests/golden/``):
the input producer (``CameraRig`` synchronisation, ``RigCalibration.get_world_extrinsics``),
the URDF rig loader, and the ``SlamPose`` quaternion conventions.
"""
