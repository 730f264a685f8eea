# Task-manager client for R model containers.
#
# Same function surface as the reference's R overlay
# (APIs/1.0/base-r/task_management/api_task.R:7-120): AddTask, UpdateTaskStatus, CompleteTask,
# FailTask, GetTaskStatus, AddPipelineTask.  It talks to this platform's HTTP store routes
# (POST /v1/cache/upsert, GET /v1/cache/get?taskId=) instead of the Azure Functions, and fixes the
# reference's undefined is.empty() and data.frame-array JSON bodies.
#
# Configuration (same variable names the Python side reads):
#   CACHE_CONNECTOR_UPSERT_URI  default http://127.0.0.1:8080/v1/cache/upsert
#   CACHE_CONNECTOR_GET_URI     default http://127.0.0.1:8080/v1/cache/get
#
# Requires the `curl` and `jsonlite` packages.  R is not installed in the build image, so this file
# is untested here ("parity unpinned"; see docs/PARITY.md).

library(curl)
library(jsonlite)

.ai4e_env <- function(name, default) {
  v <- Sys.getenv(name)
  if (nchar(v) == 0) default else v
}

.ai4e_upsert_uri <- function() .ai4e_env("CACHE_CONNECTOR_UPSERT_URI", "http://127.0.0.1:8080/v1/cache/upsert")
.ai4e_get_uri <- function() .ai4e_env("CACHE_CONNECTOR_GET_URI", "http://127.0.0.1:8080/v1/cache/get")

.ai4e_error <- function(status = "error") list(TaskId = "-1", Status = status)

.ai4e_post_task <- function(task) {
  h <- new_handle()
  handle_setheaders(h, "Content-Type" = "application/json")
  handle_setopt(h, postfields = toJSON(task, auto_unbox = TRUE, null = "null"))
  r <- curl_fetch_memory(.ai4e_upsert_uri(), handle = h)
  list(code = r$status_code, body = rawToChar(r$content))
}

GetTaskStatus <- function(taskId) {
  sep <- if (grepl("?", .ai4e_get_uri(), fixed = TRUE)) "&" else "?"
  r <- curl_fetch_memory(paste0(.ai4e_get_uri(), sep, "taskId=", URLencode(taskId, reserved = TRUE)))
  if (r$status_code != 200) {
    message(sprintf("GetTaskStatus: task %s -> HTTP %d", taskId, r$status_code))
    return(.ai4e_error())
  }
  fromJSON(rawToChar(r$content))
}

.ai4e_update <- function(taskId, status, backendStatus) {
  old <- GetTaskStatus(taskId)
  if (identical(old$TaskId, "-1")) return(old)
  endpoint <- if (is.null(old$Endpoint) || nchar(old$Endpoint) == 0) "http://localhost" else old$Endpoint
  r <- .ai4e_post_task(list(TaskId = taskId, Status = status, BackendStatus = backendStatus,
                            Endpoint = endpoint, PublishToGrid = FALSE))
  if (r$code != 200) return(list(TaskId = taskId, Status = "unable to update"))
  fromJSON(r$body)
}

# The platform creates tasks; a model container only looks up the one it was handed (taskId header).
AddTask <- function(request) {
  tid <- request$HTTP_TASKID
  if (is.null(request) || is.null(tid)) return(.ai4e_error())
  GetTaskStatus(tid)
}

UpdateTaskStatus <- function(taskId, status) .ai4e_update(taskId, status, "running")
CompleteTask <- function(taskId, status) .ai4e_update(taskId, status, "completed")
FailTask <- function(taskId, status) .ai4e_update(taskId, status, "failed")

# Re-point the task at {scheme}://{host}/{version}/{org}/{api} and publish it to that endpoint.
AddPipelineTask <- function(taskId, organization_moniker, version, api_name, body) {
  old <- GetTaskStatus(taskId)
  if (identical(old$TaskId, "-1")) return(.ai4e_error())
  m <- regmatches(old$Endpoint, regexec("^([a-zA-Z][a-zA-Z0-9+.-]*)://([^/]+)", old$Endpoint))[[1]]
  if (length(m) < 3) return(.ai4e_error())
  nxt <- sprintf("%s://%s/%s/%s/%s", m[2], m[3], version, organization_moniker, api_name)
  if (!is.null(body) && !is.character(body)) body <- as.character(toJSON(body, auto_unbox = TRUE))
  r <- .ai4e_post_task(list(TaskId = taskId, Status = "created", BackendStatus = "created",
                            Endpoint = nxt, Body = body, PublishToGrid = TRUE))
  if (r$code != 200) return(list(TaskId = taskId, Status = "not found"))
  fromJSON(r$body)
}
