"""Conformance of the fake API server (testing/fakeapi.py) with the Kubernetes API semantics
the operator relies on.

Most control-plane tests run against this fake instead of envtest's real kube-apiserver (no
Go toolchain or binaries here), so its fidelity bounds what those tests prove (SURVEY.md §7.7,
hard part 4).  Each test pins one documented apiserver behaviour; where the fake deliberately
simplifies (no strategic-merge patch; the garbage collector acts at once unless gc_delay /
foreground_hold say otherwise), the test says so.
"""

import asyncio

import pytest

from network_operator_amd.api.v1alpha1 import types as T
from network_operator_amd.operator import kube
from network_operator_amd.operator.kube import ApiClient, ApiError, KubeConfig
from network_operator_amd.testing.fakeapi import FakeApiServer

P, DS, PODS = kube.NETWORKCLUSTERPOLICIES, kube.DAEMONSETS, kube.PODS


def _run(body, **kw):
    async def wrapper():
        fake = FakeApiServer(**kw)
        url = await fake.start()
        client = ApiClient(KubeConfig(host=url))
        try:
            await body(fake, client)
        finally:
            await client.close()
            await fake.stop()

    asyncio.run(asyncio.wait_for(wrapper(), 60))


def _policy(name="p", **so):
    return T.new_policy(name, **so).to_dict()


def test_create_sets_server_fields_and_rejects_duplicates():
    async def body(fake, c):
        o = await c.create(P, _policy())
        md = o["metadata"]
        assert md["uid"] and md["creationTimestamp"] and md["generation"] == 1 and int(md["resourceVersion"]) > 0
        with pytest.raises(ApiError) as e:
            await c.create(P, _policy())
        assert e.value.status == 409 and e.value.reason == "AlreadyExists"
        with pytest.raises(ApiError) as e:
            await c.get(P, "missing")
        assert e.value.status == 404 and e.value.reason == "NotFound"
    _run(body)


def test_generation_moves_with_spec_only_and_status_is_a_subresource():
    async def body(fake, c):
        o = await c.create(P, _policy(mtu=9000))
        # metadata-only change: same generation, new resourceVersion
        o["metadata"]["labels"] = {"a": "b"}
        o2 = await c.replace(P, o)
        assert o2["metadata"]["generation"] == 1 and o2["metadata"]["resourceVersion"] != o["metadata"]["resourceVersion"]
        # spec change: generation + 1
        o2["spec"]["amdScaleOut"]["mtu"] = 4200
        o3 = await c.replace(P, o2)
        assert o3["metadata"]["generation"] == 2
        # status written through the main resource is ignored (status subresource) ...
        o3["status"] = {"targets": 7, "ready": 7, "state": "All good", "errors": []}
        o4 = await c.replace(P, o3)
        assert "status" not in o4 or o4["status"].get("targets") != 7
        # ... and spec written through /status is ignored; the generation does not move
        o4["status"] = {"targets": 1, "ready": 0, "state": "Working on it..", "errors": []}
        o4["spec"]["amdScaleOut"]["mtu"] = 1500
        o5 = await c.replace_status(P, o4)
        assert o5["status"]["targets"] == 1 and o5["spec"]["amdScaleOut"]["mtu"] == 4200
        assert o5["metadata"]["generation"] == 2
    _run(body)


def test_optimistic_concurrency_and_noop_updates():
    async def body(fake, c):
        o = await c.create(P, _policy())
        stale = dict(o, metadata=dict(o["metadata"]))
        o["metadata"]["labels"] = {"x": "1"}
        await c.replace(P, o)
        stale["metadata"]["labels"] = {"x": "2"}
        with pytest.raises(ApiError) as e:
            await c.replace(P, stale)
        assert e.value.status == 409 and e.value.reason == "Conflict"
        # an update that changes nothing keeps the resourceVersion and emits no event
        cur = await c.get(P, "p")
        n_events = len(fake.events)
        same = await c.replace(P, cur)
        assert same["metadata"]["resourceVersion"] == cur["metadata"]["resourceVersion"]
        assert len(fake.events) == n_events
    _run(body)


def test_merge_and_json_patch():
    async def body(fake, c):
        await c.create(P, _policy())
        o = await c.patch(P, "p", {"metadata": {"labels": {"k": "v"}}})
        assert o["metadata"]["labels"] == {"k": "v"}
        o = await c.patch(P, "p", {"metadata": {"labels": {"k": None}}})  # RFC 7386: null deletes
        assert not o["metadata"].get("labels")
        o = await c.patch(P, "p", [{"op": "add", "path": "/spec/logLevel", "value": 3}], patch_type="json")
        assert o["spec"]["logLevel"] == 3 and o["metadata"]["generation"] == 2
    _run(body)


def test_schema_validation_rejects_invalid_objects():
    async def body(fake, c):
        bad = _policy(mtu=100)  # below the CRD minimum
        with pytest.raises(ApiError) as e:
            await c.create(P, bad)
        assert e.value.status == 422 and e.value.reason == "Invalid"
    _run(body)


def test_list_label_selector_and_watch_resume():
    async def body(fake, c):
        a = await c.create(P, dict(_policy("a"), metadata={"name": "a", "labels": {"team": "x"}}))
        await c.create(P, dict(_policy("b"), metadata={"name": "b", "labels": {"team": "y"}}))
        lst = await c.list(P, label_selector="team=x")
        assert [i["metadata"]["name"] for i in lst["items"]] == ["a"]
        assert int(lst["metadata"]["resourceVersion"]) >= int(a["metadata"]["resourceVersion"])
        # a watch from a resourceVersion replays what happened after it, in order
        rv = lst["metadata"]["resourceVersion"]
        await c.delete(P, "b")
        seen = []
        async for typ, obj in c.watch(P, resource_version=rv, timeout_seconds=1, bookmarks=False):
            seen.append((typ, obj["metadata"]["name"]))
        assert seen == [("DELETED", "b")]
    _run(body)


def test_watch_from_a_compacted_version_is_410_gone():
    async def body(fake, c):
        o = await c.create(P, _policy())
        fake.compact()
        with pytest.raises(ApiError) as e:
            async for _ in c.watch(P, resource_version=o["metadata"]["resourceVersion"], timeout_seconds=1):
                pass
        assert e.value.status == 410
    _run(body)


def test_owner_references_cascade_in_the_background():
    async def body(fake, c):
        p = await c.create(P, _policy())
        ds = {"apiVersion": "apps/v1", "kind": "DaemonSet",
              "metadata": {"name": "d", "ownerReferences": [{"apiVersion": T.API_VERSION, "kind": T.KIND, "name": "p",
                                                             "uid": p["metadata"]["uid"], "controller": True}]},
              "spec": {"selector": {"matchLabels": {"app": "x"}},
                       "template": {"metadata": {"labels": {"app": "x"}}, "spec": {"containers": [{"name": "c"}]}}}}
        await c.create(DS, ds, namespace="ns")
        fake.add_node("n1")
        assert [pod["spec"]["nodeName"] for pod in fake.list_objects(PODS)] == ["n1"]  # DaemonSet controller
        await c.delete(P, "p")
        assert fake.get_object(DS, "d", "ns") is None  # garbage collector: dependents follow
        assert fake.list_objects(PODS) == []           # ... and theirs
    _run(body)


def test_daemonset_status_counts_matching_nodes_and_ready_pods():
    async def body(fake, c):
        ds = {"apiVersion": "apps/v1", "kind": "DaemonSet", "metadata": {"name": "d"},
              "spec": {"selector": {"matchLabels": {"app": "x"}},
                       "template": {"metadata": {"labels": {"app": "x"}},
                                    "spec": {"nodeSelector": {"gpu": "yes"}, "containers": [{"name": "c"}]}}}}
        await c.create(DS, ds, namespace="ns")
        fake.add_node("n1", {"gpu": "yes"})
        fake.add_node("n2", {"gpu": "no"})
        fake.add_node("n3", {"gpu": "yes"})
        fake.set_agent_ready("n3")
        st = (await c.get(DS, "d", "ns"))["status"]
        assert (st["desiredNumberScheduled"], st["numberReady"]) == (2, 1)
        fake.set_node_labels("n2", {"gpu": "yes"})  # a node joins the selector
        st = (await c.get(DS, "d", "ns"))["status"]
        assert st["desiredNumberScheduled"] == 3
    _run(body)


def test_list_in_chunks_with_limit_and_continue():
    async def body(fake, c):
        for i in range(7):
            await c.create(P, _policy(f"p{i}"))
        seen, cont, pages = [], "", 0
        while True:
            lst = await c.list(P, limit=3, continue_=cont)
            seen += [x["metadata"]["name"] for x in lst["items"]]
            pages += 1
            cont = lst["metadata"].get("continue", "")
            if not cont:
                break
        assert seen == [f"p{i}" for i in range(7)] and pages == 3
        assert "continue" not in (await c.list(P))["metadata"]  # no limit: one page
    _run(body)


def test_finalizers_hold_deletion_and_the_gc_respects_them():
    async def body(fake, c):
        pol = _policy()
        pol["metadata"]["finalizers"] = ["x/y"]
        p = await c.create(P, pol)
        await c.delete(P, "p")
        held = fake.get_object(P, "p")
        assert held["metadata"]["deletionTimestamp"] and held["metadata"]["finalizers"] == ["x/y"]
        held = dict(held, metadata=dict(held["metadata"], finalizers=[]))
        await c.replace(P, held)  # the last finalizer goes: so does the object
        assert fake.get_object(P, "p") is None
        assert p["metadata"]["uid"] not in fake._owned
    _run(body)


def test_foreground_deletion_waits_for_dependents_and_collects_new_ones():
    """``propagationPolicy: Foreground``: the owner gets the foregroundDeletion finalizer and a
    deletionTimestamp, the garbage collector deletes its dependents, deletes any dependent created
    while the owner waits (kubectl delete --cascade=foreground), and releases the owner once none
    is left; the owner's own finalizers still hold it after that."""
    async def body(fake, c):
        pol = _policy()
        pol["metadata"]["finalizers"] = ["x/y"]
        p = await c.create(P, pol)
        ref = [{"apiVersion": T.API_VERSION, "kind": T.KIND, "name": "p", "uid": p["metadata"]["uid"], "controller": True}]

        def job(name):
            return {"apiVersion": "batch/v1", "kind": "Job", "metadata": {"name": name, "ownerReferences": ref},
                    "spec": {"template": {"spec": {"restartPolicy": "Never", "containers": [{"name": "c"}]}}}}

        await c.create(kube.JOBS, job("before"), namespace="ns")
        await c.delete(P, "p", propagation="Foreground")
        held = fake.get_object(P, "p")
        assert held["metadata"]["deletionTimestamp"]
        assert held["metadata"]["finalizers"] == ["x/y", "foregroundDeletion"]
        assert fake.get_object(kube.JOBS, "before", "ns") is None
        created = await c.create(kube.JOBS, job("during"), namespace="ns")  # accepted, then collected
        assert created["metadata"]["name"] == "during" and fake.get_object(kube.JOBS, "during", "ns") is None
        unowned = dict(job("unowned"), metadata={"name": "unowned"})
        await c.create(kube.JOBS, unowned, namespace="ns")
        await asyncio.sleep(0.4)  # the collector releases the owner: only its own finalizer is left
        held = fake.get_object(P, "p")
        assert held["metadata"]["finalizers"] == ["x/y"]
        await c.create(kube.JOBS, job("after"), namespace="ns")  # no longer collected
        assert fake.get_object(kube.JOBS, "after", "ns") is not None
        await c.replace(P, dict(held, metadata=dict(held["metadata"], finalizers=[])))
        assert fake.get_object(P, "p") is None
        assert fake.get_object(kube.JOBS, "after", "ns") is None  # background GC once the owner is gone
        assert fake.get_object(kube.JOBS, "unowned", "ns") is not None
    _run(body, foreground_hold=0.2)


def test_a_dependent_created_after_its_owner_is_gone_is_collected():
    """The garbage collector's dangling-reference rule: a controller acting on a stale cache
    creates a DaemonSet owned by a policy deleted a moment before; it is accepted and then
    deleted.  A dependent with one live owner out of two stays."""
    async def body(fake, c):
        p = await c.create(P, _policy())
        q = await c.create(P, _policy("q"))
        ref = {"apiVersion": T.API_VERSION, "kind": T.KIND, "name": "p", "uid": p["metadata"]["uid"], "controller": True}
        await c.delete(P, "p")

        def ds(name, refs):
            return {"apiVersion": "apps/v1", "kind": "DaemonSet", "metadata": {"name": name, "ownerReferences": refs},
                    "spec": {"selector": {"matchLabels": {"app": "x"}},
                             "template": {"metadata": {"labels": {"app": "x"}}, "spec": {"containers": [{"name": "c"}]}}}}
        created = await c.create(DS, ds("late", [ref]), namespace="ns")
        assert created["metadata"]["name"] == "late"
        assert fake.get_object(DS, "late", "ns") is None
        live = {"apiVersion": T.API_VERSION, "kind": T.KIND, "name": "q", "uid": q["metadata"]["uid"]}
        await c.create(DS, ds("shared", [ref, live]), namespace="ns")
        assert fake.get_object(DS, "shared", "ns") is not None
    _run(body)
