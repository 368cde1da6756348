"""Embedded (Raft) journal wire schema.

Contract source: core/transport/src/main/proto/grpc/raft_journal.proto:1-77 (JournalQueryRequest,
SnapshotData, RaftJournalService UploadSnapshot / DownloadSnapshot) and
grpc/messaging_transport.proto (MessagingService, the tunnel the reference runs Apache Ratis
over).  The consensus RPCs themselves (vote / append / timeout-now) are Ratis-internal in the
reference; here they are first-class messages of ``alluxio.grpc.raft`` served on the embedded
journal port next to RaftJournalService.  ``SnapshotData`` carries two extra fields (100/101:
the sender's term and id) so a snapshot push doubles as Raft's InstallSnapshot.
"""

SCHEMA = r"""
package alluxio.grpc.meta
msg AddQuorumServerRequest serverAddress=1:alluxio.grpc.NetAddress
msg GetSnapshotInfoRequest
msg SnapshotMetadata snapshotTerm=1:i64 snapshotIndex=2:i64
msg GetSnapshotInfoResponse latest=1:SnapshotMetadata
msg GetSnapshotRequest
msg JournalQueryRequest snapshotInfoRequest=1:GetSnapshotInfoRequest snapshotRequest=2:GetSnapshotRequest
    addQuorumServerRequest=3:AddQuorumServerRequest
msg JournalQueryResponse snapshotInfoResponse=1:GetSnapshotInfoResponse
msg SnapshotData snapshotTerm=1:i64 snapshotIndex=2:i64 chunk=3:bytes offset=4:i64 eof=5:bool
    leaderTerm=100:i64 leaderId=101:str
msg UploadSnapshotPRequest data=1:SnapshotData
msg UploadSnapshotPResponse offsetReceived=1:i64
msg DownloadSnapshotPRequest offsetReceived=1:i64
msg DownloadSnapshotPResponse data=1:SnapshotData
rpc RaftJournalService UploadSnapshot *UploadSnapshotPRequest *UploadSnapshotPResponse
rpc RaftJournalService DownloadSnapshot *DownloadSnapshotPRequest *DownloadSnapshotPResponse

package alluxio.grpc.messaging
msg MessagingRequestHeader requestId=1:i64
msg MessagingResponseHeader requestId=1:i64 isThrowable=2:bool
msg TransportMessage requestHeader=1:MessagingRequestHeader responseHeader=2:MessagingResponseHeader
    message=3:bytes
rpc MessagingService connect *TransportMessage *TransportMessage

package alluxio.grpc.raft
msg RaftNamedEntry master=1:str entry=2:alluxio.proto.journal.JournalEntry
msg RaftCommand entries=1:RaftNamedEntry* peers=2:str* primaryStart=3:i64
msg RaftLogEntry term=1:i64 index=2:i64 command=3:bytes
msg RaftSnapshotHeader index=1:i64 term=2:i64 peers=3:str* nextSequenceNumber=4:i64 masters=5:str*
msg RequestVotePRequest term=1:i64 candidateId=2:str lastLogIndex=3:i64 lastLogTerm=4:i64
    preVote=5:bool transfer=6:bool
msg RequestVotePResponse term=1:i64 granted=2:bool
msg AppendEntriesPRequest term=1:i64 leaderId=2:str prevLogIndex=3:i64 prevLogTerm=4:i64
    entries=5:RaftLogEntry* leaderCommit=6:i64
msg AppendEntriesPResponse term=1:i64 success=2:bool matchIndex=3:i64 conflictIndex=4:i64
msg TimeoutNowPRequest term=1:i64 leaderId=2:str
msg TimeoutNowPResponse accepted=1:bool
rpc RaftServerService RequestVote RequestVotePRequest RequestVotePResponse
rpc RaftServerService AppendEntries AppendEntriesPRequest AppendEntriesPResponse
rpc RaftServerService TimeoutNow TimeoutNowPRequest TimeoutNowPResponse
rpc RaftServerService JournalQuery alluxio.grpc.meta.JournalQueryRequest alluxio.grpc.meta.JournalQueryResponse
"""
