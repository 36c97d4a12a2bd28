"""TEST INFRASTRUCTURE ONLY — CPU oracle for the nff-go ACL hot path.

rules_oracle: independent Python restatement of the rule parser
              (packet/acl.go:121-411, go1.13 stdlib semantics).
oracle:       ctypes front of acl_oracle.c, the literal restatement of
              (*Packet).l3ACL (packet/acl.go:508-565, packet/packet.go:233-363).
Never imported by the product (nff-go_amd/); only by tests/, smoke() and the
cpu_baseline leg of bench.py.
"""
