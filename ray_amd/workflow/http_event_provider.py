"""HTTP events for workflows (reference: python/ray/workflow/http_event_provider.py).

``HTTPEventProvider`` is a Serve application (route prefix ``/event``) that external
systems POST events to: ``POST /event/send_event/<workflow_id>`` with JSON
``{"event_key": ..., "event_payload": ...}``. ``HTTPListener`` is the EventListener a
``workflow.wait_for_event(HTTPListener, event_key=...)`` step uses: it registers
(workflow id, event key) with the provider and waits for the matching POST. The POST is
answered only after the workflow has checkpointed the event:

* 200 — the event was delivered to the waiting step and checkpointed;
* 404 — no step of that workflow is waiting for that key (or the JSON lacks a field);
* 500 — the step reported that checkpointing failed.

Pending registrations and acknowledgements are keyed by (workflow id, event key), so two
workflows may use the same key. The provider keeps its state in one replica's memory: a
provider restart drops registrations (the waiting steps then never see their events; the
reference has the same limitation).
"""

# (no postponed annotations here: FastAPI must see the real `Request` type of send_event's
# parameter through Serve's ingress wrapper, or it treats `req` as a query parameter)
import asyncio

from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse

from ray_amd import serve
from ray_amd.workflow.api import EventListener, get_current_task_id, get_current_workflow_id

HTTP_EVENT_PROVIDER_NAME = "WorkflowHTTPEventProvider"


class WorkflowEventHandleError(Exception):
    """An HTTP event could not be handled (duplicate registration, unknown ack)."""

    def __init__(self, workflow_id: str, what: str):
        super().__init__(f"Workflow[id={workflow_id}] HTTP event handling failed: {what}")


app = FastAPI()


@serve.deployment(num_replicas=1)
@serve.ingress(app)
class HTTPEventProvider:
    def __init__(self):
        self.waiting = {}  # (workflow id, key) -> Future of (key, payload)
        self.acks = {}     # (workflow id, key) -> Future of bool (checkpointed)

    @app.post("/send_event/{workflow_id}")
    async def send_event(self, workflow_id: str, req: Request):
        body = await req.json()
        if not isinstance(body, dict) or "event_key" not in body or \
                "event_payload" not in body:
            return JSONResponse(status_code=404, content={"error": {
                "code": 404, "message": "the JSON body needs event_key and event_payload"}})
        key = (workflow_id, body["event_key"])
        fut = self.waiting.get(key)
        if fut is None or fut.done():
            return JSONResponse(status_code=404, content={"error": {
                "code": 404, "message": "no workflow step is waiting for this workflow_id "
                                        "and event_key; register before sending"}})
        ack = self.acks[key] = asyncio.get_running_loop().create_future()
        fut.set_result((body["event_key"], body["event_payload"]))
        try:
            ok = await ack
        finally:
            self.acks.pop(key, None)
            self.waiting.pop(key, None)
        if ok:
            return JSONResponse(status_code=200, content={})
        return JSONResponse(status_code=500, content={"error": {
            "code": 500, "message": "the workflow failed to checkpoint the event"}})

    async def get_event_payload(self, workflow_id: str, event_key: str):
        key = (workflow_id, event_key)
        if key in self.waiting and not self.waiting[key].done():
            raise WorkflowEventHandleError(workflow_id,
                                           f"event key {event_key!r} already registered")
        fut = self.waiting[key] = asyncio.get_running_loop().create_future()
        return await fut

    async def report_checkpointed(self, workflow_id: str, event_key: str,
                                  confirmation: bool) -> str:
        ack = self.acks.get((workflow_id, event_key))
        if ack is None:
            raise WorkflowEventHandleError(
                workflow_id, f"no pending HTTP request for event key {event_key!r} (the "
                             "provider may have restarted)")
        if not ack.done():
            ack.set_result(bool(confirmation))
        return "OK"


def start_http_event_provider():
    """Deploy the provider (idempotent) and return its handle."""
    try:
        return serve.get_app_handle(HTTP_EVENT_PROVIDER_NAME)
    except Exception:  # noqa: BLE001  (not deployed yet)
        return serve.run(HTTPEventProvider.bind(), name=HTTP_EVENT_PROVIDER_NAME,
                         route_prefix="/event")


class HTTPListener(EventListener):
    """EventListener for HTTPEventProvider events. ``event_key`` defaults to the waiting
    step's task id; the event is ``(event_key, event_payload)``."""

    def __init__(self):
        self.handle = start_http_event_provider()
        self.workflow_id = None
        self.event_key = None

    async def poll_for_event(self, event_key: str | None = None):
        self.workflow_id = get_current_workflow_id()
        self.event_key = event_key if event_key is not None else get_current_task_id()
        return await self.handle.get_event_payload.remote(self.workflow_id, self.event_key)

    async def event_checkpointed(self, event) -> None:
        await self.handle.report_checkpointed.remote(self.workflow_id, self.event_key, True)
