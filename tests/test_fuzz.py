"""Fuzzing the control plane (the reference fuzzes CR fields against a live cluster and
watches the operator log for crashes: reference test/fuzz/fuzz_test.go, README.md:3-8).

Here the oracle is stronger: random create / update / delete sequences with random (valid
and invalid) specs go through the fake API server (schema validation included) while the
real controller runs; afterwards every surviving policy has exactly one DaemonSet whose agent
arguments equal ``agent_args(policy)``, no DaemonSet outlives its policy, and every worker
is still alive.
"""

import asyncio
import os

from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from network_operator_amd.api.v1alpha1 import types as T
from network_operator_amd.operator import kube
from network_operator_amd.operator.controller import PolicyController
from network_operator_amd.operator.kube import ApiClient, ApiError, KubeConfig
from network_operator_amd.operator.reconciler import agent_args, host_nic_agent_args
from network_operator_amd.testing.fakeapi import FakeApiServer

NS = "fuzz"

def mostly(valid, invalid):
    """Values that are valid three times in four: the churn reaches the reconciler, and the
    invalid ones still exercise admission."""
    return st.one_of(st.sampled_from(valid), st.sampled_from(valid), st.sampled_from(valid), st.sampled_from(invalid))


mtu = mostly([1500, 4200, 9000], [0, 1000, 10000])
so_strategy = st.fixed_dictionaries({}, optional={
    "layer": mostly(["L2", "L3"], ["L3BGP", ""]),
    "mtu": mtu,
    "image": st.sampled_from(["amd/x:1", "registry.local/agent@sha256:abc"]),
    "pullPolicy": mostly(["Always", "Never", "IfNotPresent"], ["", "Sometimes"]),
    "disableNetworkManager": st.booleans(),
    "xgmiCheck": st.booleans(),
    "lldpAnnounce": st.booleans(),
    # round 3 / 4 fields
    "disableFirmwareLldp": st.booleans(),
    "handDcbxToHost": st.booleans(),
    "allowPolicyRouted": st.booleans(),
    "checkPeerMtu": st.booleans(),
    "keepConfigOnRestart": st.booleans(),
    "minLinkSpeedGbps": mostly([0, 100, 400], [-1]),
    "lldpWait": mostly(["2m", "90s"], ["", "0s", "soon"]),
    "railSwitchPattern": mostly(["leaf-r{rail}-.*", "spine[0-9]+"], ["(?i)leaf", "("]),
    "interfaces": st.lists(mostly(["ens1np0", "ens2np0"], ["bad name", ""]), max_size=2, unique=True),
    "nicDrivers": st.lists(st.sampled_from(["mlx5_core", "bnxt_en"]), max_size=2, unique=True),
    "rcclEnv": st.dictionaries(mostly(["NCCL_IB_TC", "RCCL_X"], ["PATH"]), mostly(["1", "106"], ["a\nb"]),
                               max_size=2),
})
host_nic_strategy = st.fixed_dictionaries({"layer": mostly(["L2", "L3"], [""])}, optional={
    "mtu": mtu,
    "interfaces": st.lists(mostly(["ens9np0", "ens49np1"], ["x/y"]), max_size=2, unique=True),
    "nicDrivers": st.lists(st.sampled_from(["mlx5_core", "ionic"]), max_size=2, unique=True),
    "includeGpuRails": st.booleans(),
    "allowPolicyRouted": st.booleans(),
    "checkPeerMtu": st.booleans(),
    "keepConfigOnRestart": st.booleans(),
    "verifyPeers": st.booleans(),
    "lldpWait": mostly(["45s"], ["forever"]),
})
spec_strategy = st.fixed_dictionaries({
    "configurationType": st.sampled_from(["amd-so", "amd-so", "amd-so", "host-nic"]),
    "amdScaleOut": so_strategy,
    "nodeSelector": st.dictionaries(st.sampled_from(["a", "b/c", "amd.feature.node.kubernetes.io/gpu-ready"]),
                                    st.sampled_from(["true", "x"]), min_size=1, max_size=2)
                    | st.just({}),
}, optional={"logLevel": st.integers(-1, 9), "hostNic": host_nic_strategy,
             "tolerations": st.lists(mostly([{"key": "amd.com/gpu", "operator": "Exists", "effect": "NoSchedule"},
                                             {"key": "dedicated", "operator": "Equal", "value": "gpu"}],
                                            [{"operator": "Exists", "value": "x"}, {"key": "a b"}]), max_size=2),
             "priorityClassName": mostly(["system-node-critical", "gpu-infra"], ["Bad_Name"])})
op_strategy = st.tuples(st.sampled_from(["create", "update", "delete"]), st.sampled_from(["p0", "p1", "p2"]), spec_strategy)


# NETOP_FUZZ_EXAMPLES raises the count for a longer soak (`NETOP_FUZZ_EXAMPLES=200 make fuzz`).
@settings(max_examples=int(os.environ.get("NETOP_FUZZ_EXAMPLES", "12")), deadline=None,
          suppress_health_check=[HealthCheck.too_slow])
@given(ops=st.lists(op_strategy, min_size=1, max_size=12))
def test_random_policy_churn_converges(ops):
    async def body():
        fake = FakeApiServer()
        url = await fake.start()
        client = ApiClient(KubeConfig(host=url))
        ctl = PolicyController(client, NS, workers=3, record_events=False)
        await ctl.start()
        try:
            for op, name, spec in ops:
                try:
                    if op == "create":
                        await client.create(kube.NETWORKCLUSTERPOLICIES, {"apiVersion": T.API_VERSION, "kind": T.KIND,
                                                                           "metadata": {"name": name}, "spec": spec})
                    elif op == "update":
                        cur = await client.get(kube.NETWORKCLUSTERPOLICIES, name)
                        cur["spec"] = spec
                        await client.replace(kube.NETWORKCLUSTERPOLICIES, cur)
                    else:
                        await client.delete(kube.NETWORKCLUSTERPOLICIES, name)
                except ApiError as e:
                    assert e.status in (404, 409, 422), e
                await asyncio.sleep(0.005)  # 5 ms apart, like the reference fuzzer

            async def converged():
                pols = {p["metadata"]["name"]: p for p in fake.list_objects(kube.NETWORKCLUSTERPOLICIES)}
                dss = {d["metadata"]["name"]: d for d in fake.list_objects(kube.DAEMONSETS)}
                assert set(dss) <= set(pols), "orphan DaemonSet"
                for name, p in pols.items():
                    pol = T.NetworkClusterPolicy.from_dict(p)
                    want = {T.CONFIG_AMD_SCALE_OUT: agent_args, T.CONFIG_HOST_NIC: host_nic_agent_args}.get(
                        pol.spec.configurationType)
                    if want is None:
                        continue  # unknown types never get a DaemonSet (they error and back off)
                    assert name in dss, f"no DaemonSet for {name}"
                    assert dss[name]["spec"]["template"]["spec"]["containers"][0]["args"] == want(pol)
                    assert p.get("status", {}).get("state") == "No targets"
                return True

            end = asyncio.get_event_loop().time() + 20  # generous: CI runs this beside netns scenarios
            while True:
                try:
                    await converged()
                    break
                except AssertionError:
                    if asyncio.get_event_loop().time() > end:
                        raise
                    await asyncio.sleep(0.05)
            assert all(not t.done() for t in ctl._tasks), "a controller task died"
        finally:
            await ctl.stop()
            await client.close()
            await fake.stop()

    asyncio.run(asyncio.wait_for(body(), 60))
