# Round 6, timing only (wrong output): the packed kernel without its record
# loads (every lane XORs zeros) -- what the chunk loads cost the launch
EDITS = [
    ("sg_pack.hip", """            d0 = pld16(src); d1 = pld16(src + 16); d2 = pld16(src + 32); d3 = pld16(src + 48);""",
     """            asm volatile("" :: "v"(src));"""),
]
