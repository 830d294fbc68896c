"""Offer recommendations: wrappers around Mesos offer operations.

Reference: sdk/.../offer/{Reserve,Unreserve,Create,Destroy,Launch,StoreTaskInfo}OfferRecommendation
.java and UninstallRecommendation.java. ``StoreTaskInfoRecommendation`` carries no Mesos operation;
it is persisted (write-ahead) by the launch recorder before the ACCEPT is sent.
"""
from __future__ import annotations

from typing import Optional

from dcos_commons_amd.mesos import protos as P

Op = P.Offer.Operation


class OfferRecommendation:
    __slots__ = ("offer", "operation")

    def __init__(self, offer: P.Offer, operation: Optional[P.Offer.Operation]):
        self.offer = offer
        self.operation = operation

    def get_operation(self) -> Optional[P.Offer.Operation]:
        return self.operation

    @property
    def offer_id(self) -> P.OfferID:
        return self.offer.id

    @property
    def agent_id(self) -> P.AgentID:
        return self.offer.agent_id

    def __repr__(self):
        t = Op.Type.Name(self.operation.type) if self.operation is not None else "NONE"
        return f"{type(self).__name__}({t}, agent={self.offer.agent_id.value})"


class UninstallRecommendation(OfferRecommendation):
    __slots__ = ("resource",)


class ReserveOfferRecommendation(OfferRecommendation):
    __slots__ = ()

    def __init__(self, offer: P.Offer, resource: P.Resource):
        op = Op(type=Op.RESERVE)
        r = op.reserve.resources.add()  # copied once, straight into the operation
        r.CopyFrom(resource)
        if r.HasField("disk") and r.disk.HasField("source"):
            r.disk.ClearField("persistence")
            r.disk.ClearField("volume")
        else:
            r.ClearField("disk")
        r.ClearField("revocable")
        super().__init__(offer, op)


class UnreserveOfferRecommendation(UninstallRecommendation):
    __slots__ = ()

    def __init__(self, offer: P.Offer, resource: P.Resource):
        r = P.Resource()
        r.CopyFrom(resource)
        if resource.HasField("disk") and resource.disk.HasField("source"):
            src = P.Resource.DiskInfo.Source()
            src.CopyFrom(resource.disk.source)
            r.ClearField("disk")
            r.disk.source.CopyFrom(src)
        else:
            r.ClearField("disk")
            r.ClearField("revocable")
        op = Op(type=Op.UNRESERVE)
        op.unreserve.resources.add().CopyFrom(r)
        super().__init__(offer, op)
        self.resource = r


class CreateOfferRecommendation(OfferRecommendation):
    __slots__ = ()

    def __init__(self, offer: P.Offer, resource: P.Resource):
        op = Op(type=Op.CREATE)
        op.create.volumes.add().CopyFrom(resource)
        super().__init__(offer, op)


class DestroyOfferRecommendation(UninstallRecommendation):
    __slots__ = ()

    def __init__(self, offer: P.Offer, resource: P.Resource):
        r = P.Resource()
        r.CopyFrom(resource)
        r.ClearField("revocable")
        op = Op(type=Op.DESTROY)
        op.destroy.volumes.add().CopyFrom(r)
        super().__init__(offer, op)
        self.resource = resource


class LaunchOfferRecommendation(OfferRecommendation):
    __slots__ = ()

    def __init__(self, offer: P.Offer, task_info: P.TaskInfo, executor_info: P.ExecutorInfo):
        op = Op(type=Op.LAUNCH_GROUP)
        op.launch_group.executor.CopyFrom(executor_info)
        op.launch_group.task_group.tasks.add().CopyFrom(task_info)
        super().__init__(offer, op)

    @property
    def task_info(self) -> P.TaskInfo:
        return self.operation.launch_group.task_group.tasks[0]

    @property
    def executor_info(self) -> P.ExecutorInfo:
        return self.operation.launch_group.executor


class StoreTaskInfoRecommendation(OfferRecommendation):
    __slots__ = ("task_info", "executor_info")

    def __init__(self, offer: P.Offer, task_info: P.TaskInfo, executor_info: P.ExecutorInfo):
        super().__init__(offer, None)
        self.task_info = task_info
        self.executor_info = executor_info

    def state_store_task_info(self) -> P.TaskInfo:
        t = P.TaskInfo()
        t.CopyFrom(self.task_info)
        t.executor.CopyFrom(self.executor_info)
        return t
