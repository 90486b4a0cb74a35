"""Shim of ``isaaclab.utils.pretrained_checkpoint``: no published checkpoints offline."""


def get_published_pretrained_checkpoint(workflow: str, task_name: str):
    print(f"[WARN] no published pre-trained checkpoint for {task_name} ({workflow}) in the MI355X build")
    return None
