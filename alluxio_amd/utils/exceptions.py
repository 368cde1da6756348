"""Status exceptions with gRPC status-code mapping.

Mirrors the reference's ``AlluxioStatusException`` hierarchy
(core/base/src/main/java/alluxio/exception/status/AlluxioStatusException.java) so that an error
raised on the master or worker crosses the wire as the same gRPC status code a Java client
expects, and is re-raised as the same exception type on our client side.
"""
from __future__ import annotations

import enum


class Status(enum.IntEnum):
    # gRPC canonical codes (grpc.StatusCode values)
    OK = 0
    CANCELLED = 1
    UNKNOWN = 2
    INVALID_ARGUMENT = 3
    DEADLINE_EXCEEDED = 4
    NOT_FOUND = 5
    ALREADY_EXISTS = 6
    PERMISSION_DENIED = 7
    RESOURCE_EXHAUSTED = 8
    FAILED_PRECONDITION = 9
    ABORTED = 10
    OUT_OF_RANGE = 11
    UNIMPLEMENTED = 12
    INTERNAL = 13
    UNAVAILABLE = 14
    DATA_LOSS = 15
    UNAUTHENTICATED = 16


class AlluxioStatusException(Exception):
    status: Status = Status.UNKNOWN

    def __init__(self, message: str = "", cause: BaseException | None = None):
        super().__init__(message)
        self.message = message
        self.__cause__ = cause

    @classmethod
    def from_status(cls, status: int, message: str) -> "AlluxioStatusException":
        klass = _BY_STATUS.get(Status(status), UnknownException)
        return klass(message)


class CancelledException(AlluxioStatusException):
    status = Status.CANCELLED


class UnknownException(AlluxioStatusException):
    status = Status.UNKNOWN


class InvalidArgumentException(AlluxioStatusException):
    status = Status.INVALID_ARGUMENT


class DeadlineExceededException(AlluxioStatusException):
    status = Status.DEADLINE_EXCEEDED


class NotFoundException(AlluxioStatusException):
    status = Status.NOT_FOUND


class AlreadyExistsException(AlluxioStatusException):
    status = Status.ALREADY_EXISTS


class PermissionDeniedException(AlluxioStatusException):
    status = Status.PERMISSION_DENIED


class ResourceExhaustedException(AlluxioStatusException):
    status = Status.RESOURCE_EXHAUSTED


class FailedPreconditionException(AlluxioStatusException):
    status = Status.FAILED_PRECONDITION


class AbortedException(AlluxioStatusException):
    status = Status.ABORTED


class OutOfRangeException(AlluxioStatusException):
    status = Status.OUT_OF_RANGE


class UnimplementedException(AlluxioStatusException):
    status = Status.UNIMPLEMENTED


class InternalException(AlluxioStatusException):
    status = Status.INTERNAL


class UnavailableException(AlluxioStatusException):
    status = Status.UNAVAILABLE


class DataLossException(AlluxioStatusException):
    status = Status.DATA_LOSS


class UnauthenticatedException(AlluxioStatusException):
    status = Status.UNAUTHENTICATED


_BY_STATUS = {c.status: c for c in (
    CancelledException, UnknownException, InvalidArgumentException, DeadlineExceededException,
    NotFoundException, AlreadyExistsException, PermissionDeniedException,
    ResourceExhaustedException, FailedPreconditionException, AbortedException,
    OutOfRangeException, UnimplementedException, InternalException, UnavailableException,
    DataLossException, UnauthenticatedException)}


# Domain-specific aliases used across master / worker code (reference alluxio.exception.*).
class FileDoesNotExistException(NotFoundException):
    pass


class FileAlreadyExistsException(AlreadyExistsException):
    pass


class DirectoryNotEmptyException(FailedPreconditionException):
    pass


class InvalidPathException(InvalidArgumentException):
    pass


class BlockDoesNotExistException(NotFoundException):
    pass


class BlockAlreadyExistsException(AlreadyExistsException):
    pass


class WorkerOutOfSpaceException(ResourceExhaustedException):
    pass


class InvalidWorkerStateException(FailedPreconditionException):
    pass


class FileIncompleteException(FailedPreconditionException):
    pass


class AccessControlException(PermissionDeniedException):
    pass


class JournalClosedException(UnavailableException):
    pass


class ConnectionFailedException(UnavailableException):
    pass


class UfsException(UnavailableException):
    pass


def wrap(exc: BaseException) -> AlluxioStatusException:
    """Convert arbitrary exceptions into a status exception (reference ``AlluxioStatusException.fromThrowable``)."""
    if isinstance(exc, AlluxioStatusException):
        return exc
    if isinstance(exc, FileNotFoundError):
        return NotFoundException(str(exc), exc)
    if isinstance(exc, FileExistsError):
        return AlreadyExistsException(str(exc), exc)
    if isinstance(exc, PermissionError):
        return PermissionDeniedException(str(exc), exc)
    if isinstance(exc, (ValueError, TypeError)):
        return InvalidArgumentException(str(exc), exc)
    if isinstance(exc, TimeoutError):
        return DeadlineExceededException(str(exc), exc)
    if isinstance(exc, (ConnectionError, OSError)):
        return UnavailableException(str(exc), exc)
    return UnknownException(f"{type(exc).__name__}: {exc}", exc)
