"""Literal Python restatement of the reference PartitionStateMachine (small cases only).

Follows mq-broker/src/main/java/metadata/raft/PartitionStateMachine.java line by line:
  messages: List<String>               (:26)   -> list of bytes
  consumerOffsets: Map<String, Long>   (:27)   -> dict
  handleMessageAppendRequest           (:64-69) messages.addAll(request.getMessages())
  handleConsumerOffsetUpdateRequest    (:71-77) consumerOffsets.put(id, offset)
  handleBatchRead                      (:85-110) off = getOrDefault(id, 0);
                                                 messages[off, min(off + max, size)), offset = off
  getConsumerOffset                    (:112-119)
and the client loops that drive it:
  PartitionClient.sendMessage wraps ONE message per MessageAppendRequest
  (mq-common/src/main/java/partition/selector/PartitionClient.java:39-40);
  ConsumerClientImpl.consume reads max 10 then commits offset + n
  (mq-common/src/main/java/client/ConsumerClientImpl.java:21,87-109).
It has no Raft: every applied entry is committed (the reference only applies committed entries).
"""
from __future__ import annotations


class PartitionStateMachine:
    def __init__(self, group_id: str):
        self.group_id = group_id
        self.messages: list[bytes] = []
        self.consumer_offsets: dict[str, int] = {}

    def handle_message_append_request(self, messages: list[bytes]) -> None:
        self.messages.extend(messages)

    def handle_consumer_offset_update_request(self, consumer_id: str, offset: int) -> None:
        self.consumer_offsets[consumer_id] = offset

    def handle_batch_read(self, consumer_id: str, max_messages: int) -> tuple[list[bytes], int]:
        offset = self.consumer_offsets.get(consumer_id, 0)
        end = min(offset + max_messages, len(self.messages))
        return [self.messages[i] for i in range(offset, end)], offset

    def get_consumer_offset(self, consumer_id: str) -> int:
        return self.consumer_offsets.get(consumer_id, 0)


class Broker:
    """groupId = topic + "-" + partitionId -> state machine (PartitionManager.activePartitions)."""

    def __init__(self, topic: str, partitions: int):
        self.topic = topic
        self.sms = [PartitionStateMachine(f"{topic}-{p}") for p in range(partitions)]

    def produce(self, pid: int, message: bytes) -> int:
        sm = self.sms[pid]
        off = len(sm.messages)
        sm.handle_message_append_request([message])
        return off

    def consume(self, pid: int, consumer_id: str, max_messages: int = 10) -> tuple[list[bytes], int]:
        msgs, off = self.sms[pid].handle_batch_read(consumer_id, max_messages)
        self.sms[pid].handle_consumer_offset_update_request(consumer_id, off + len(msgs))
        return msgs, off
