"""Resource requests / managers (reference: python/ray/air/tests/
test_resource_manager_fixed.py, test_resource_manager_placement_group.py) and
job_submission JobType / DriverInfo."""
import pytest

import ray_amd as ray
from ray_amd.air import ResourceRequest
from ray_amd.air.execution import FixedResourceManager, PlacementGroupResourceManager


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def test_request_head_bundle_and_equality():
    r = ResourceRequest([{"CPU": 0}, {"CPU": 1, "GPU": 0}, {"CPU": 2}], strategy="SPREAD")
    assert r.head_bundle_is_empty and r.head_cpus == 0
    assert r.bundles == [{"CPU": 1}, {"CPU": 2}] and r.required_resources == {"CPU": 3}
    assert r == ResourceRequest([{}, {"CPU": 1}, {"CPU": 2}], strategy="SPREAD")
    assert len({r, ResourceRequest([{}, {"CPU": 1}, {"CPU": 2}], strategy="SPREAD")}) == 1
    with pytest.raises(ValueError):
        ResourceRequest([{"CPU": 1}], strategy="NOPE")


def test_fixed_manager_bookkeeping():
    m = FixedResourceManager({"CPU": 4})
    big, small = ResourceRequest([{"CPU": 3}]), ResourceRequest([{"CPU": 2}])
    m.request_resources(big)
    m.request_resources(small)
    assert m.has_resources_ready(big)
    a = m.acquire_resources(big)
    assert a is not None and not m.has_resources_ready(small)  # 1 CPU left
    m.free_resources(a)
    assert m.has_resources_ready(small)
    with pytest.raises(ValueError):
        import pickle

        pickle.dumps(m)


def test_placement_group_manager_annotates_actors(cluster):
    m = PlacementGroupResourceManager(update_interval_s=0.0)
    req = ResourceRequest([{"CPU": 1}, {"CPU": 1}])
    m.request_resources(req)
    ray.get(m.get_resource_futures(), timeout=30)
    assert m.has_resources_ready(req)
    acq = m.acquire_resources(req)

    @ray.remote
    class A:
        def pg(self):
            return ray.get_runtime_context().get_placement_group_id()

    head, worker = acq.annotate_remote_entities([A, A])
    a, b = head.remote(), worker.remote()
    pgid = acq.placement_group.id.hex()
    assert ray.get(a.pg.remote()) == pgid and ray.get(b.pg.remote()) == pgid
    ray.kill(a)
    ray.kill(b)
    m.free_resources(acq)
    m.clear()
    # an unsatisfiable request never becomes ready
    huge = ResourceRequest([{"CPU": 64}])
    m.request_resources(huge)
    m.update_state()
    assert not m.has_resources_ready(huge)
    m.cancel_resource_request(huge)


def test_job_type_and_driver_info():
    from ray_amd.job_submission import DriverInfo, JobDetails, JobType

    d = JobDetails.from_dict({"submission_id": "s", "entrypoint": "python x.py",
                              "status": "RUNNING", "type": "DRIVER", "driver_pid": 42,
                              "job_id": "01000000"})
    assert d.type is JobType.DRIVER and d.type == "DRIVER"
    assert d.driver_info == DriverInfo(id="01000000", node_ip_address="127.0.0.1", pid="42")
