// Golden vectors for the OBJ parser's number semantics (wpt_obj.cpp):
// obj_parser.ts:3-51 calls JavaScript's parseFloat / parseInt and stores the
// results in a Float32Array. This script asks the JS engine itself (node,
// no reference code) for those results on edge-case strings; f64 values are
// written as hex bits, f32 (Math.fround) likewise.
// Run: node tests/golden/make_obj_golden.js > tests/golden/obj_numbers.json
const floats = ['1', '-0', '+1.5', '.5', '5.', '.', '', ' 7', '\t8', '1e3', '1e', '1e+', '1E-2x', 'Infinity',
  '-Infinity', '+Infinity', 'inf', 'nan', 'NaN', '0x10', '0X1f', '1_000', '12abc', '  -3.25e1 ',
  '1.7976931348623157e309', '4.9e-325', '0.1', '3.4028235677973366e38', '3.4028236e38', '1.00000005960464477539',
  '1.0000000596046448', '00012', '-.25', '1.5e-45', '7.006e-46', '\r5', '5\r', '2.5e+2.5', '-', '+', 'e5',
  '0.30000000000000004', '123456789012345678901234567890', '9007199254740993', '1e-310'];
const ints = ['1', '2/5', '0x2', '0X3', '-1', '+2', ' 3', '3abc', '', 'x', '1.9', '1e2', '0x', '08', '0b1',
  '007', '-0x10', '\t4', '5\r', '99', '0', '-0'];
const hex64 = x => Buffer.from(new Float64Array([x]).buffer).toString('hex');
const hex32 = x => Buffer.from(new Float32Array([x]).buffer).toString('hex');
const out = {
  note: 'parseFloat / parseInt / Math.fround of node ' + process.version + '; values as little-endian hex bits',
  floats: floats.map(s => ({s, f64: hex64(parseFloat(s)), f32: hex32(Math.fround(parseFloat(s)))})),
  ints: ints.map(s => ({s, f64: hex64(parseInt(s))})),
};
console.log(JSON.stringify(out, null, 1));
