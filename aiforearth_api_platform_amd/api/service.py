"""``APIService`` — the drop-in-model decorator API (signature-compatible with the reference).

Reference: ``APIs/1.0/base-py/ai4e_service.py:43-213``.  Kept verbatim:

* ``APIService(flask_app, logger)``; ``.api_async_func`` / ``.api_sync_func`` with parameters
  ``(api_path, methods, request_processing_function=None, maximum_concurrent_requests=None,
  content_types=None, content_max_length=None, trace_name=None)`` (``:103-109``);
* the user function receives ``func``, ``api_path``, the ``request_processing_function`` dict,
  ``taskId`` (async) and ``request`` (``:80-91,181``);
* routes ``GET {API_PREFIX}/`` (health, ``'Health check OK'``) and ``GET {API_PREFIX}/task/<id>``;
* async responses are the plain text ``'TaskId: <id>'`` (``:94``) — or the task JSON when the
  client sends ``Accept: application/json`` (the gateway form, ``request_policy.xml:23-28``);
* failures: ``FailTask(taskId, 'Task failed - try again')`` (``:185-213``).

Intended behaviour where the reference is broken (survey Appendix B #1-#5), documented here:

* admission control looks up the *full* (prefixed) path, so it actually runs with ``API_PREFIX``;
* ``maximum_concurrent_requests=None`` means unbounded (reference: TypeError);
* busy -> **429** (retryable by the dispatcher), draining -> **503**, bad content type -> 401,
  too large -> 413;
* ``DISABLE_CURRENT_REQUEST_METRIC`` is parsed as a bool, and counters are lock-protected;
* ``tracer`` falls back to the platform tracer when the logger has none;
* SIGINT *and* SIGTERM start the drain (reference handler raised TypeError on ``str + int``);
* async work runs on a bounded worker pool, not one OS thread per request, and gets a snapshot
  of the request (the Flask ``request`` proxy is invalid outside the request context).
"""
from __future__ import annotations

import concurrent.futures as cf
import json
import signal
import sys
import threading
from functools import wraps
from typing import Any, Callable, Dict, Optional

from ..config import get_config
from ..utils.metrics import REGISTRY, current_requests_key
from ..utils.tracing import get_tracer
from .task_manager import TaskManager

MAX_REQUESTS_KEY_NAME = "max_requests"
CONTENT_TYPE_KEY_NAME = "content_types"
CONTENT_MAX_KEY_NAME = "content_max_length"


class RequestSnapshot:
    """Thread-safe copy of the parts of a Flask request a model function uses."""

    def __init__(self, req):
        self.headers = dict(req.headers)
        self.args = req.args.to_dict() if hasattr(req.args, "to_dict") else dict(req.args)
        self.path = req.path
        self.url = req.url
        self.method = req.method
        self.content_type = req.content_type
        self.content_length = req.content_length
        self.data = req.get_data()
        self.files = {k: v.read() for k, v in req.files.items()} if getattr(req, "files", None) else {}

    def get_data(self):
        return self.data

    def get_json(self, force: bool = False, silent: bool = False):
        try:
            return json.loads(self.data or b"null")
        except ValueError:
            if silent:
                return None
            raise

    @property
    def json(self):
        return self.get_json(silent=True)


class APIService:
    def __init__(self, flask_app, logger, task_manager: Optional[TaskManager] = None, max_workers: int = 32,
                 install_signal_handlers: bool = True):
        from flask import request  # noqa: F401  (Flask is the compat host, as in the reference)

        cfg = get_config()
        self.app = flask_app
        self.log = logger
        self.cfg = cfg
        self.is_terminating = False
        self.func_properties: Dict[str, Dict[str, Any]] = {}
        self.func_request_counts: Dict[str, int] = {}
        self._count_mu = threading.Lock()
        self.api_prefix = cfg.api_prefix or ""
        self.tracer = getattr(logger, "tracer", None) or get_tracer()
        self.api_task_manager = task_manager or TaskManager()
        self.executor = cf.ThreadPoolExecutor(max_workers=max_workers, thread_name_prefix="ai4e-async")
        self._inflight: set = set()
        if install_signal_handlers and threading.current_thread() is threading.main_thread():
            signal.signal(signal.SIGINT, self.initialize_term)
            signal.signal(signal.SIGTERM, self.initialize_term)

        self.app.add_url_rule(self.api_prefix + "/", endpoint="ai4e_health", view_func=self.health_check,
                              methods=["GET"])
        self.app.add_url_rule(self.api_prefix + "/task/<id>", endpoint="ai4e_task", view_func=self.task_status,
                              methods=["GET"])
        self.app.before_request(self.before_request)

    # ------------------------------------------------------------------ routes
    def health_check(self):
        return "Health check OK"

    def task_status(self, id):
        st = self.api_task_manager.GetTaskStatus(str(id))
        return {"TaskId": id, "Status": st.get("Status"), "Timestamp": st.get("Timestamp"),
                "Endpoint": st.get("Endpoint", "uri")}

    # ------------------------------------------------------------------ decorators
    def api_func(self, is_async, api_path, methods, request_processing_function, maximum_concurrent_requests,
                 content_types=None, content_max_length=None, trace_name=None, *args, **kwargs):
        from flask import request

        full_path = self.api_prefix + api_path

        def decorator_api_func(func):
            if full_path not in self.func_properties:
                self.func_properties[full_path] = {MAX_REQUESTS_KEY_NAME: maximum_concurrent_requests,
                                                   CONTENT_TYPE_KEY_NAME: content_types,
                                                   CONTENT_MAX_KEY_NAME: content_max_length}
                self.func_request_counts[api_path] = 0

            @wraps(func)
            def api(*a, **kw):
                internal_args = {"func": func, "api_path": api_path}
                if request_processing_function:
                    return_values = request_processing_function(request) or {}
                    combined = {**internal_args, **kw, **return_values}
                else:
                    combined = {**internal_args, **kw}
                if is_async:
                    task_info = self.api_task_manager.AddTask(request)
                    task_id = str(task_info["TaskId"])
                    combined["taskId"] = task_id
                    self.wrap_async_endpoint(trace_name, *a, **combined)
                    if "application/json" in (request.headers.get("Accept") or ""):
                        return self.api_task_manager.GetTaskStatus(task_id)
                    return "TaskId: " + task_id
                return self.wrap_sync_endpoint(trace_name, *a, **combined)

            api.__name__ = "api_" + api_path.replace("/", "")
            self.app.add_url_rule(full_path, endpoint=api.__name__, view_func=api, methods=methods,
                                  provide_automatic_options=True)
            return func

        return decorator_api_func

    def api_async_func(self, api_path, methods, request_processing_function=None, maximum_concurrent_requests=None,
                       content_types=None, content_max_length=None, trace_name=None, *args, **kwargs):
        return self.api_func(True, api_path, methods, request_processing_function, maximum_concurrent_requests,
                             content_types, content_max_length, trace_name, *args, **kwargs)

    def api_sync_func(self, api_path, methods, request_processing_function=None, maximum_concurrent_requests=None,
                      content_types=None, content_max_length=None, trace_name=None, *args, **kwargs):
        return self.api_func(False, api_path, methods, request_processing_function, maximum_concurrent_requests,
                             content_types, content_max_length, trace_name, *args, **kwargs)

    # ------------------------------------------------------------------ drain + admission
    def initialize_term(self, signum, frame):
        print(f"Signal handler called with signal: {signum}. Service is terminating and will no longer "
              "accept requests.", file=sys.stderr)
        self.is_terminating = True

    def before_request(self):
        from flask import abort, request

        if self.is_terminating:
            abort(503, {"message": "Service is terminating, please try again later."})
        props = self.func_properties.get(request.path)
        if props is None:
            return None
        api_path = request.path[len(self.api_prefix):] if self.api_prefix else request.path
        mx = props[MAX_REQUESTS_KEY_NAME]
        if mx is not None:
            with self._count_mu:
                busy = self.func_request_counts.get(api_path, 0) + 1 > mx
            if busy:
                abort(429, {"message": "Service is busy, please try again later."})
        cts = props[CONTENT_TYPE_KEY_NAME]
        if cts and request.content_type not in cts:
            abort(401, {"message": "Content-type must be " + str(cts)})
        cmax = props[CONTENT_MAX_KEY_NAME]
        if cmax and (request.content_length or 0) > cmax:
            abort(413, {"message": "Request content too large (" + str(request.content_length)
                        + "). Must be smaller than: " + str(cmax)})
        return None

    # ------------------------------------------------------------------ counters
    def update_processing_count(self, api_path, increment_by, decrement_by):
        payload = {"ApiPath": self.api_prefix + api_path, "ServiceCluster": self.cfg.service_cluster,
                   "IncrementBy": increment_by, "DecrementBy": decrement_by}
        if self.cfg.current_processing_upsert_uri:
            import requests

            try:
                requests.post(self.cfg.current_processing_upsert_uri, data=json.dumps(payload), timeout=5)
            except Exception as e:  # metric push must never fail the request
                self.log.log_exception(e)
        else:
            from ..gateway.control import get_control_plane

            get_control_plane().current_processing_upsert(payload)

    def _adjust(self, api_path, delta):
        with self._count_mu:
            self.func_request_counts[api_path] = self.func_request_counts.get(api_path, 0) + delta
            v = self.func_request_counts[api_path]
        REGISTRY.gauge(current_requests_key(self.cfg.service_cluster, self.api_prefix + api_path)).set(v)
        if not self.cfg.disable_current_request_metric:
            self.update_processing_count(api_path, max(delta, 0), max(-delta, 0))

    def increment_requests(self, api_path):
        self._adjust(api_path, +1)

    def decrement_requests(self, api_path):
        self._adjust(api_path, -1)

    # ------------------------------------------------------------------ execution
    def wrap_sync_endpoint(self, trace_name=None, *args, **kwargs):
        with self.tracer.span(name=trace_name or kwargs["api_path"]):
            return self._execute_func_with_counter(False, *args, **kwargs)

    def wrap_async_endpoint(self, trace_name=None, *args, **kwargs):
        with self.tracer.span(name=trace_name or kwargs["api_path"]):
            self._create_and_execute_thread(*args, **kwargs)

    def _create_and_execute_thread(self, *args, **kwargs):
        from flask import request

        kwargs["request"] = RequestSnapshot(request)
        # Count the request as in flight from admission, so max-concurrency sees queued work too.
        self.increment_requests(kwargs["api_path"])
        fut = self.executor.submit(self._execute_func_with_counter, True, *args, _counted=True, **kwargs)
        self._inflight.add(fut)
        fut.add_done_callback(self._inflight.discard)

    def _log_and_fail_exception(self, is_async, **kwargs):
        task_id = kwargs.get("taskId")
        self.log.log_exception(sys.exc_info()[0], task_id or "")
        if is_async and task_id:
            self.api_task_manager.FailTask(task_id, "Task failed - try again")

    def _execute_func_with_counter(self, is_async=True, *args, _counted=False, **kwargs):
        from flask import abort
        from werkzeug.exceptions import HTTPException

        func = kwargs["func"]
        api_path = kwargs["api_path"]
        if not _counted:
            self.increment_requests(api_path)
        try:
            return func(*args, **kwargs)
        except HTTPException as e:
            self._log_and_fail_exception(is_async, **kwargs)
            return e
        except Exception:
            self._log_and_fail_exception(is_async, **kwargs)
            if is_async:
                return None
            abort(500)
        finally:
            self.decrement_requests(api_path)

    def wait_idle(self, timeout: Optional[float] = None) -> bool:
        """Block until all async work has finished (graceful drain helper)."""
        done, not_done = cf.wait(list(self._inflight), timeout=timeout)
        return not not_done
