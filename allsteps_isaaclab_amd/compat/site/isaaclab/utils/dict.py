"""Shim of ``isaaclab.utils.dict.print_dict``."""


def print_dict(val, nesting: int = -4, start: bool = True) -> None:
    if isinstance(val, dict):
        if not start:
            print("")
        nesting += 4
        for k, v in val.items():
            print(nesting * " " + str(k) + ": ", end="")
            print_dict(v, nesting, start=False)
    else:
        print(val)
