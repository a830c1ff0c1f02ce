"""Disk BSSRDFs on the device beyond the golden renders (test_gpu_parity.py
covers sss_disk*, sss_blur at BVH widths 2/4/8): the load-time refusal of
the one combination the device does not take."""
import pytest

from raytracingproject_amd import scene as sc
from raytracingproject_amd import scenes

pytestmark = pytest.mark.gpu


def test_disk_bssrdf_in_a_volume_scene_is_refused_at_load():
    """Disk BSSRDFs with volumes would need the exit points' volume stack
    updates (kernel_path_subsurface.h:84-95): load_kernels names the feature
    instead of rendering something else."""
    from raytracingproject_amd.device import DeviceError, HIPDevice

    s = scenes.sss_disk_cornell(16, 16, 1)
    s.world_volume = sc.volume_scatter((0.8, 0.8, 0.8), density=0.001)
    ds = sc.compile_scene(s)
    assert ds.data.integrator.use_volumes
    dev = HIPDevice(0)
    try:
        with pytest.raises(DeviceError, match="disk BSSRDFs"):
            dev.upload_scene(ds)
    finally:
        dev.close()
