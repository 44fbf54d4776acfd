"""CPU oracle for the reference's decision semantics -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package, as the checker (or the timed CPU baseline); the product path never does.
"""
